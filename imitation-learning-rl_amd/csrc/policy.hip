// policy.hip - on-GPU inference of the reference's PPO policy network and a device-resident rollout loop
// (the sampler's policy.compute_actions -> env.step loop with no host round trip).
//
// Network (train_config.py:107-111, RLlib 1.2 FullyConnectedNetwork with fcnet_hiddens [256, 256],
// fcnet_activation tanh, free_log_std True): mean = W3 tanh(W2 tanh(W1 obs + b1) + b2) + b3, action distribution
// DiagGaussian(mean, exp(log_std)); RLlib's clip_actions clips the sample to the Box [-1, 1] before env.step.
// Weights are fp32 [in][out] (the TF kernel layout RLlib's get_weights() returns).  Two shapes are in use: the
// low-level policy 70 -> 17 and the hierarchical env's high-level policy 44 -> 2 (train_config.py:23-27, 262-298:
// the same FCNet on the 44-dim high observation and the 2-dim heading action); any n_in <= 72, n_out <= 32 works.
//
// MI355X mapping: one block = 16 envs x 16 waves (1024 threads; 4096 envs = 256 blocks = one per CU, four waves
// per SIMD); batches of >= 64 K rows (a fragment's SampleBatch columns) take 64 rows per block, each wave reusing its
// weight fragments over four 16-row tiles (157 KB of LDS: one block per CU, a quarter of the weight traffic per row).  Wave w owns the 16x16 output tile of columns 16w..16w+15 of each hidden layer (waves 0, 1 the two
// tiles of the 17-wide output layer), computed on v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain).
// Weights are re-laid out once at hum_policy_create into MFMA B-fragment order (per tile, per 4 k-steps, per lane
// a float4), so a wave fetches a whole layer's operands with coalesced 16-byte loads issued before the first
// MFMA that needs them; activations go through LDS at a row pitch that keeps the A-fragment reads
// conflict-free (pitch = 2 mod 32 banks).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>

#include "../../include/humanoid_env.h"

void hum_internal_set_error(const char* msg);
int hum_internal_device(const hum_env* env);   // humanoid_env.hip
int hum_internal_rollout_fused(hum_env* e, const float* pw, uint64_t seed, int32_t k, int32_t explore, uint64_t step0,
                               float* obs, float* obs_reset, uint8_t* done, float* reward, float* act_last,
                               float* obs_traj, float* act_traj, float* rew_traj, uint8_t* done_traj,
                               float* mean_traj, void* stream);
int hum_internal_hier_step_acted(hum_env* e, const float* high_act, const float* low_act, uint8_t* agents,
                                 float* high_obs, float* low_obs, float* high_rew, float* low_rew, uint8_t* done,
                                 uint32_t flags, float* high_obs_reset, uint8_t* acted, void* stream);
int hum_internal_hier_rollout_fused(hum_env* e, const float* pw_high, uint64_t seed_high, const float* pw_low,
                                    uint64_t seed_low, int32_t k, int32_t explore, uint64_t step0, const hum_hier_io* io,
                                    const hum_hier_traj* T, float* mean_high, float* mean_low, void* stream);

namespace {

constexpr int H = 256, K1 = 72;   // K1: the largest input (70) padded to a multiple of 4; inputs n_in <= K1
constexpr int MAX_OUT = 32;         // outputs n_out <= two 16-wide tiles
constexpr int ROWS = 16, WAVES = H / 16;
// B-fragment layout: [tile][k-step quad][lane][4]; k-steps per layer 18 (K1 / 4, quads padded to 5), 64, 64
constexpr int SQ1 = 5, SQ2 = 16, SQ3 = 16, NT3 = 2;
constexpr size_t FRAG1 = (size_t)WAVES * SQ1 * 64 * 4, FRAG2 = (size_t)WAVES * SQ2 * 64 * 4, FRAG3 = (size_t)NT3 * SQ3 * 64 * 4;
constexpr int PX = 98, PH = 258;   // LDS row pitches (floats): 2 mod 32, so the 32 lanes of a b32 read hit 32 banks

struct PolicyArgs {
    const float* f1; const float* f2; const float* f3;   // B fragments (frag_layout)
    const float* w1; const float* b1; const float* w2; const float* b2; const float* w3; const float* b3;
    const float* log_std;
    const float* obs; const float* obs_reset; const unsigned char* done;
    float* act; float* mean_out; float* obs_in_out; float* raw_out;
    int n, explore, n_in, n_out;
    unsigned long long seed, step;
};

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// B fragment of k-step s for lane l of a 16-column tile at column c0 of W[K x ncol] (row stride ldw):
// W[4s + (l >> 4)][c0 + (l & 15)], 0 outside the matrix
__host__ inline float frag_value(const float* W, int K, int ldw, int ncol, int c0, int s, int l) {
    const int k = 4 * s + (l >> 4), c = c0 + (l & 15);
    return k < K && c < ncol ? W[(size_t)k * ldw + c] : 0.f;
}
__host__ inline void frag_layout(const float* W, int K, int ldw, int ncol, int ntile, int nsq, float* out) {
    for (int t = 0; t < ntile; t++)
        for (int q = 0; q < nsq; q++)
            for (int l = 0; l < 64; l++)
                for (int j = 0; j < 4; j++)
                    out[(((size_t)t * nsq + q) * 64 + l) * 4 + j] = frag_value(W, K, ldw, ncol, 16 * t, 4 * q + j, l);
}

// the wave's B fragments of one layer (tile t), every load issued at once
template <int NSQ>
__device__ inline void load_frags(const float* __restrict__ F, int t, f32x4* b) {
    const int l = threadIdx.x & 63;
    const f32x4* src = reinterpret_cast<const f32x4*>(F) + (size_t)t * NSQ * 64 + l;
#pragma unroll
    for (int q = 0; q < NSQ; q++) b[q] = src[q * 64];
}
// RT independent 16x16 tiles acc[rt] = X[rt 16 .. rt 16 + 15][0 .. 4 NS) (LDS, pitch ldx) times the tile's fragments;
// each tile's k-steps in order (the k-ordered fp32 fma chain the fused kernels restate), the RT chains interleaved so
// consecutive MFMAs do not wait on each other's results
template <int NS, int RT>
__device__ inline void mfma_tiles(const float* X, int ldx, const f32x4* b, f32x4 (&acc)[RT]) {
    const int l = threadIdx.x & 63;
    const float* xr = X + (l & 15) * ldx + (l >> 4);
#pragma unroll
    for (int rt = 0; rt < RT; rt++) acc[rt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; s++)
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
            acc[rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(xr[rt * ROWS * ldx + 4 * s], b[s >> 2][s & 3], acc[rt], 0, 0, 0);
}

// RT row tiles of 16 per block: every wave reuses its B fragments over the RT tiles (RT = 4 for large batches:
// a quarter of the L2 weight traffic per row; RT = 1 keeps one 16-row block per CU for a 4096-lane step)
template <int RT>
__global__ void __launch_bounds__(64 * WAVES) policy_kernel(PolicyArgs p) {
    constexpr int NR = ROWS * RT;
    __shared__ float xs[NR * PX];
    __shared__ float h1[NR * PH];
    __shared__ float h2[NR * PH];
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63;
    const int row0 = blockIdx.x * NR;
    // every fragment this wave needs, before anything waits (hidden layers: tile = wave; output layer: waves 0, 1)
    f32x4 b1f[SQ1], b2f[SQ2];
    load_frags<SQ1>(p.f1, wave, b1f);
    load_frags<SQ2>(p.f2, wave, b2f);
    // observation tile (done lanes read their post-reset observation: the sampler's next input)
    for (int e = tid; e < NR * K1; e += blockDim.x) {
        const int r = e / K1, k = e - r * K1, i = row0 + r;
        float v = 0.f;
        if (i < p.n && k < p.n_in) {
            const bool rs = p.obs_reset && p.done && p.done[i];
            v = (rs ? p.obs_reset : p.obs)[(long)i * p.n_in + k];
        }
        xs[r * PX + k] = v;
        if (p.obs_in_out && i < p.n && k < p.n_in) p.obs_in_out[(long)i * p.n_in + k] = v;
    }
    __syncthreads();
    const int c = 16 * wave + (l & 15);   // C/D map: lane l, register q -> row 4 (l >> 4) + q, column l & 15
    {
        const float bias = p.b1[c];
        f32x4 acc[RT];
        mfma_tiles<K1 / 4, RT>(xs, PX, b1f, acc);
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int q = 0; q < 4; q++) h1[(rt * ROWS + 4 * (l >> 4) + q) * PH + c] = tanhf(acc[rt][q] + bias);
    }
    __syncthreads();
    {
        const float bias = p.b2[c];
        f32x4 acc[RT];
        mfma_tiles<H / 4, RT>(h1, PH, b2f, acc);
#pragma unroll
        for (int rt = 0; rt < RT; rt++)
#pragma unroll
            for (int q = 0; q < 4; q++) h2[(rt * ROWS + 4 * (l >> 4) + q) * PH + c] = tanhf(acc[rt][q] + bias);
    }
    __syncthreads();
    if (wave < NT3 && 16 * wave < p.n_out) {   // output layer: up to two 16-wide tiles of columns, one per wave
        f32x4 b3f[SQ3];
        load_frags<SQ3>(p.f3, wave, b3f);
        f32x4 oo[RT];
        mfma_tiles<H / 4, RT>(h2, PH, b3f, oo);
#pragma unroll
        for (int rt = 0; rt < RT; rt++) {
            const f32x4 o = oo[rt];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = rt * ROWS + 4 * (l >> 4) + q, c3 = 16 * wave + (l & 15), i = row0 + r;
                if (c3 < p.n_out && i < p.n) {
                    const float mean = o[q] + p.b3[c3];
                    float a = mean;
                    if (p.explore) {   // DiagGaussian sample: mean + exp(log_std) * N(0, 1), counter-based Box-Muller
                        // (seed, lane, step, column) each through its own mixing round: no two triples share a draw
                        const unsigned long long x = mix64(mix64(mix64(p.seed ^ (unsigned long long)i) ^ p.step) ^ (unsigned long long)c3);
                        const float u1 = ((float)(x >> 40) + 1.f) * 0x1.0p-24f;   // (0, 1]
                        const float u2 = (float)((x >> 16) & 0xFFFFFFull) * 0x1.0p-24f;
                        a = mean + expf(p.log_std[c3]) * sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
                    }
                    const long o2 = (long)i * p.n_out + c3;
                    p.act[o2] = fminf(fmaxf(a, -1.f), 1.f);   // clip_actions (Box [-1, 1])
                    if (p.raw_out) p.raw_out[o2] = a;           // the sample itself (SampleBatch actions)
                    if (p.mean_out) p.mean_out[o2] = mean;
                }
            }
        }
    }
}

}  // namespace

struct hum_policy {
    int device;
    int n_in, n_out;
    float* w;   // one allocation: w1 b1 w2 b2 w3 b3 log_std, then the B fragments of w1, w2, w3
    const float *w1, *b1, *w2, *b2, *w3, *b3, *log_std, *f1, *f2, *f3;
    unsigned long long seed;
};

namespace {
int perr(int code, const std::string& m) {
    hum_internal_set_error(m.c_str());
    return code;
}
}  // namespace

extern "C" {

int hum_policy_create(int32_t device, const float* w1, const float* b1, const float* w2, const float* b2,
                      const float* w3, const float* b3, const float* log_std, uint64_t seed, hum_policy** out) {
    return hum_policy_create_ex(device, HUM_NOBS, HUM_NACT, w1, b1, w2, b2, w3, b3, log_std, seed, out);
}

int hum_policy_create_ex(int32_t device, int32_t n_in, int32_t n_out, const float* w1, const float* b1, const float* w2,
                         const float* b2, const float* w3, const float* b3, const float* log_std, uint64_t seed,
                         hum_policy** out) {
    if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !out) return perr(HUM_ERR_ARG, "hum_policy_create: null argument");
    if (n_in < 1 || n_in > K1 || n_out < 1 || n_out > MAX_OUT)
        return perr(HUM_ERR_ARG, "hum_policy_create: n_in must be in [1, 72] and n_out in [1, 32]");
    if (hipSetDevice(device) != hipSuccess) return perr(HUM_ERR_HIP, "hum_policy_create: hipSetDevice");
    // w1 is stored padded to K1 rows (rows n_in .. 71 zero) so the kernel's k loop needs no bound; the block layout
    // (w1 [72][256], b1, w2, b2, w3 [256][n_out], b3, log_std) is what hum_rollout_fused's in-kernel network reads
    const size_t n1 = (size_t)K1 * H, n2 = (size_t)H * H, n3 = (size_t)H * n_out;
    const size_t nw = (n1 + H + n2 + H + n3 + n_out + n_out + 63) / 64 * 64;   // fragments 16-byte aligned
    const size_t total = nw + FRAG1 + FRAG2 + FRAG3;
    hum_policy* p = new hum_policy();
    p->device = device;
    p->n_in = n_in;
    p->n_out = n_out;
    p->seed = seed;
    if (hipMalloc((void**)&p->w, total * sizeof(float)) != hipSuccess) {
        delete p;
        return perr(HUM_ERR_HIP, "hum_policy_create: hipMalloc");
    }
    float* h = new float[total]();
    std::memcpy(h, w1, (size_t)n_in * H * sizeof(float));
    size_t o = n1;
    std::memcpy(h + o, b1, H * sizeof(float)); o += H;
    std::memcpy(h + o, w2, n2 * sizeof(float)); o += n2;
    std::memcpy(h + o, b2, H * sizeof(float)); o += H;
    std::memcpy(h + o, w3, n3 * sizeof(float)); o += n3;
    std::memcpy(h + o, b3, n_out * sizeof(float)); o += n_out;
    if (log_std) std::memcpy(h + o, log_std, n_out * sizeof(float));
    frag_layout(w1, n_in, H, H, WAVES, SQ1, h + nw);
    frag_layout(w2, H, H, H, WAVES, SQ2, h + nw + FRAG1);
    frag_layout(w3, H, n_out, n_out, NT3, SQ3, h + nw + FRAG1 + FRAG2);
    const hipError_t st = hipMemcpy(p->w, h, total * sizeof(float), hipMemcpyHostToDevice);
    delete[] h;
    if (st != hipSuccess) {
        (void)hipFree(p->w);
        delete p;
        return perr(HUM_ERR_HIP, "hum_policy_create: hipMemcpy");
    }
    p->w1 = p->w; p->b1 = p->w1 + n1; p->w2 = p->b1 + H; p->b2 = p->w2 + n2; p->w3 = p->b2 + H;
    p->b3 = p->w3 + n3; p->log_std = p->b3 + n_out;
    p->f1 = p->w + nw; p->f2 = p->f1 + FRAG1; p->f3 = p->f2 + FRAG2;
    *out = p;
    return HUM_OK;
}

int hum_policy_destroy(hum_policy* p) {
    if (!p) return HUM_OK;
    (void)hipSetDevice(p->device);
    (void)hipFree(p->w);
    delete p;
    return HUM_OK;
}

int hum_policy_act(hum_policy* p, const float* obs, const float* obs_reset, const uint8_t* done, int32_t n,
                   float* actions, float* mean_out, float* obs_in_out, int32_t explore, uint64_t step, void* stream) {
    return hum_policy_act_ex(p, obs, obs_reset, done, n, actions, mean_out, obs_in_out, nullptr, explore, step, stream);
}

int hum_policy_act_ex(hum_policy* p, const float* obs, const float* obs_reset, const uint8_t* done, int32_t n,
                      float* actions, float* mean_out, float* obs_in_out, float* raw_out, int32_t explore, uint64_t step,
                      void* stream) {
    if (!p || !obs || !actions || n <= 0) return perr(HUM_ERR_ARG, "hum_policy_act: bad argument");
    if ((obs_reset == nullptr) != (done == nullptr)) return perr(HUM_ERR_ARG, "hum_policy_act: obs_reset needs done");
    if (hipSetDevice(p->device) != hipSuccess) return perr(HUM_ERR_HIP, "hum_policy_act: hipSetDevice");
    PolicyArgs a;
    a.f1 = p->f1; a.f2 = p->f2; a.f3 = p->f3;
    a.w1 = p->w1; a.b1 = p->b1; a.w2 = p->w2; a.b2 = p->b2; a.w3 = p->w3; a.b3 = p->b3; a.log_std = p->log_std;
    a.obs = obs; a.obs_reset = obs_reset; a.done = done; a.act = actions; a.mean_out = mean_out; a.obs_in_out = obs_in_out;
    a.raw_out = raw_out;
    a.n = n; a.explore = explore; a.seed = p->seed; a.step = step; a.n_in = p->n_in; a.n_out = p->n_out;
    // batches of 4 row tiles per block once there are at least 4 such blocks per CU (the batched SampleBatch columns
    // over a fragment's k x n rows); a step's 4096 rows keep one 16-row block per CU
    if (n >= 4 * ROWS * 4 * 256)
        hipLaunchKernelGGL(policy_kernel<4>, dim3((n + 4 * ROWS - 1) / (4 * ROWS)), dim3(64 * WAVES), 0,
                           (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(policy_kernel<1>, dim3((n + ROWS - 1) / ROWS), dim3(64 * WAVES), 0, (hipStream_t)stream, a);
    const hipError_t st = hipGetLastError();
    if (st != hipSuccess) return perr(HUM_ERR_HIP, std::string("hum_policy_act: ") + hipGetErrorString(st));
    return HUM_OK;
}

// k sampler steps on the env's lanes with no host round trip: policy (on the current observation; lanes that
// finished an episode in the previous step act on their reset observation) -> hum_step with auto-reset.
// Trajectory outputs (device, any may be NULL): obs_traj [k,n,70] the policy's inputs, act_traj [k,n,17] the
// sampled actions before clip_actions (what RLlib's SampleBatch records and PPO's likelihood ratio is evaluated on;
// the env receives their clip to [-1, 1]), rew_traj [k,n], done_traj [k,n].  obs / obs_reset / done / reward are the
// env-step buffers (device [n,70], [n,70], [n], [n]); on entry obs holds the current observation and done the
// previous step's flags (zeros after a reset).  Launches go to `stream` in order.
int hum_rollout(hum_env* env, hum_policy* p, int32_t k, int32_t explore, uint64_t step0, float* obs, float* obs_reset,
                uint8_t* done, float* reward, float* act_buf, float* obs_traj, float* act_traj, float* rew_traj,
                uint8_t* done_traj, void* stream) {
    if (!env || !p || k <= 0 || !obs || !obs_reset || !done || !reward || !act_buf)
        return perr(HUM_ERR_ARG, "hum_rollout: bad argument");
    if (p->n_in != HUM_NOBS || p->n_out != HUM_NACT)
        return perr(HUM_ERR_ARG, "hum_rollout: the policy must map the 70-dim observation to the 17 actions");
    if (hum_internal_device(env) != p->device)
        return perr(HUM_ERR_ARG, "hum_rollout: the env handle and the policy are on different devices");
    const int n = hum_num_lanes(env);
    hipStream_t s = (hipStream_t)stream;
    for (int t = 0; t < k; t++) {
        int rc = hum_policy_act_ex(p, obs, obs_reset, done, n, act_buf, nullptr,
                                   obs_traj ? obs_traj + (size_t)t * n * HUM_NOBS : nullptr,
                                   act_traj ? act_traj + (size_t)t * n * HUM_NACT : nullptr, explore,
                                   step0 + (uint64_t)t, stream);
        if (rc != HUM_OK) return rc;
        rc = hum_step(env, act_buf, obs, reward, done, nullptr, HUM_STEP_AUTORESET, obs_reset, stream);
        if (rc != HUM_OK) return rc;
        if (rew_traj && hipMemcpyAsync(rew_traj + (size_t)t * n, reward, (size_t)n * sizeof(float),
                                       hipMemcpyDeviceToDevice, s) != hipSuccess)
            return perr(HUM_ERR_HIP, "hum_rollout: reward copy");
        if (done_traj && hipMemcpyAsync(done_traj + (size_t)t * n, done, (size_t)n, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return perr(HUM_ERR_HIP, "hum_rollout: done copy");
    }
    return HUM_OK;
}

int hum_rollout_fused_ex(hum_env* env, hum_policy* p, int32_t k, int32_t explore, uint64_t step0, float* obs,
                         float* obs_reset, uint8_t* done, float* reward, float* act_buf, float* obs_traj,
                         float* act_traj, float* rew_traj, uint8_t* done_traj, float* mean_traj, void* stream) {
    if (!env || !p || k <= 0 || !obs || !obs_reset || !done || !reward || !act_buf)
        return perr(HUM_ERR_ARG, "hum_rollout_fused: bad argument");
    if (p->n_in != HUM_NOBS || p->n_out != HUM_NACT)
        return perr(HUM_ERR_ARG, "hum_rollout_fused: the policy must map the 70-dim observation to the 17 actions");
    if (hum_internal_device(env) != p->device)
        return perr(HUM_ERR_ARG, "hum_rollout_fused: the env handle and the policy are on different devices");
    return hum_internal_rollout_fused(env, p->w, p->seed, k, explore, step0, obs, obs_reset, done, reward, act_buf,
                                      obs_traj, act_traj, rew_traj, done_traj, mean_traj, stream);
}

int hum_rollout_fused(hum_env* env, hum_policy* p, int32_t k, int32_t explore, uint64_t step0, float* obs,
                      float* obs_reset, uint8_t* done, float* reward, float* act_buf, float* obs_traj, float* act_traj,
                      float* rew_traj, uint8_t* done_traj, void* stream) {
    return hum_rollout_fused_ex(env, p, k, explore, step0, obs, obs_reset, done, reward, act_buf, obs_traj, act_traj,
                                rew_traj, done_traj, nullptr, stream);
}

}  // extern "C"
namespace {
// the argument checks hum_hier_rollout and hum_hier_rollout_fused share
int hier_rollout_check(const char* fn, hum_env* env, hum_policy* high, hum_policy* low, int32_t k, const hum_hier_io* io) {
    const std::string f(fn);
    if (!env || !high || !low || k <= 0 || !io) return perr(HUM_ERR_ARG, f + ": bad argument");
    if (!io->obs_high || !io->obs_high_reset || !io->obs_low || !io->done || !io->agents || !io->rew_high ||
        !io->rew_low || !io->act_high || !io->act_low)
        return perr(HUM_ERR_ARG, f + ": every hum_hier_io buffer is required");
    if (high->n_in != HUM_NOBS_HIGH || high->n_out != HUM_NACT_HIGH || low->n_in != HUM_NOBS || low->n_out != HUM_NACT)
        return perr(HUM_ERR_ARG, f + ": needs a (44, 2) high-level and a (70, 17) low-level policy");
    if (hum_internal_device(env) != high->device || hum_internal_device(env) != low->device)
        return perr(HUM_ERR_ARG, f + ": the env handle and the policies are on different devices");
    return HUM_OK;
}
}  // namespace
extern "C" {

int hum_hier_rollout(hum_env* env, hum_policy* high, hum_policy* low, int32_t k, int32_t explore, uint64_t step0,
                     const hum_hier_io* io, const hum_hier_traj* tr, void* stream) {
    if (const int rc = hier_rollout_check("hum_hier_rollout", env, high, low, k, io)) return rc;
    const hum_hier_traj none = {};
    const hum_hier_traj& T = tr ? *tr : none;
    const size_t n = (size_t)hum_num_lanes(env);
    hipStream_t s = (hipStream_t)stream;
    // per transition: the step's agents / rewards / done go straight into the trajectory rows when recorded (every
    // lane's are written when the agent is each lane's expected one), and the next transition reads done from there
    const uint8_t* done_prev = io->done;
    for (int t = 0; t < k; t++) {
        const size_t r = (size_t)t * n;
        int rc = hum_policy_act_ex(high, io->obs_high, io->obs_high_reset, done_prev, (int32_t)n, io->act_high, nullptr,
                                   T.obs_high ? T.obs_high + r * HUM_NOBS_HIGH : nullptr,
                                   T.act_high ? T.act_high + r * HUM_NACT_HIGH : nullptr, explore, step0 + (uint64_t)t,
                                   stream);
        if (rc != HUM_OK) return rc;
        rc = hum_policy_act_ex(low, io->obs_low, nullptr, nullptr, (int32_t)n, io->act_low, nullptr,
                               T.obs_low ? T.obs_low + r * HUM_NOBS : nullptr,
                               T.act_low ? T.act_low + r * HUM_NACT : nullptr, explore, step0 + (uint64_t)t, stream);
        if (rc != HUM_OK) return rc;
        uint8_t* ag = T.agents ? T.agents + r : io->agents;
        float* rh = T.rew_high ? T.rew_high + r : io->rew_high;
        float* rl = T.rew_low ? T.rew_low + r : io->rew_low;
        uint8_t* dn = T.done ? T.done + r : io->done;
        rc = hum_internal_hier_step_acted(env, io->act_high, io->act_low, ag, io->obs_high, io->obs_low, rh, rl, dn,
                                          HUM_STEP_AUTORESET, io->obs_high_reset, T.acted ? T.acted + r : nullptr, stream);
        if (rc != HUM_OK) return rc;
        done_prev = dn;
    }
    // the last transition's rows into the env buffers (when they went to the trajectory)
    const size_t last = (size_t)(k - 1) * n;
    struct { void* dst; const void* src; size_t bytes; } cp[4] = {
        {io->agents, T.agents ? T.agents + last : nullptr, n}, {io->rew_high, T.rew_high ? T.rew_high + last : nullptr, 4 * n},
        {io->rew_low, T.rew_low ? T.rew_low + last : nullptr, 4 * n}, {io->done, T.done ? T.done + last : nullptr, n}};
    for (auto& c : cp)
        if (c.src && hipMemcpyAsync(c.dst, c.src, c.bytes, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return perr(HUM_ERR_HIP, "hum_hier_rollout: copy of the last transition's rows");
    return HUM_OK;
}

// hum_hier_rollout in one launch: both networks inside the cooperative kernel's step loop, each evaluated only for
// the envs that act with it (a wave whose four envs all expect the low agent skips the high network and vice versa)
int hum_hier_rollout_fused_ex(hum_env* env, hum_policy* high, hum_policy* low, int32_t k, int32_t explore,
                              uint64_t step0, const hum_hier_io* io, const hum_hier_traj* tr, float* mean_high,
                              float* mean_low, void* stream) {
    if (const int rc = hier_rollout_check("hum_hier_rollout_fused", env, high, low, k, io)) return rc;
    const hum_hier_traj none = {};
    return hum_internal_hier_rollout_fused(env, high->w, high->seed, low->w, low->seed, k, explore, step0, io,
                                           tr ? tr : &none, mean_high, mean_low, stream);
}

int hum_hier_rollout_fused(hum_env* env, hum_policy* high, hum_policy* low, int32_t k, int32_t explore, uint64_t step0,
                           const hum_hier_io* io, const hum_hier_traj* tr, void* stream) {
    return hum_hier_rollout_fused_ex(env, high, low, k, explore, step0, io, tr, nullptr, nullptr, stream);
}

}  // extern "C"
