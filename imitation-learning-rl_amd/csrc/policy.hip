// policy.hip - on-GPU inference of the reference's PPO policy network and a device-resident rollout loop
// (the sampler's policy.compute_actions -> env.step loop with no host round trip).
//
// Network (train_config.py:107-111, RLlib 1.2 FullyConnectedNetwork with fcnet_hiddens [256, 256],
// fcnet_activation tanh, free_log_std True): mean = W3 tanh(W2 tanh(W1 obs + b1) + b2) + b3, action distribution
// DiagGaussian(mean, exp(log_std)); RLlib's clip_actions clips the sample to the Box [-1, 1] before env.step.
// Weights are fp32 [in][out] (the TF kernel layout RLlib's get_weights() returns).
//
// MI355X mapping: one 256-thread block = 16 envs x 4 waves.  Layer outputs are 16x16 tiles of
// v_mfma_f32_16x16x4_f32 (exact fp32: a k-ordered fmaf chain), each wave owning a 64-column slice of the layer;
// activations go through LDS (16 x 256 fp32 = 16 KB), weights stream from L2 (349 KB in all, resident).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <string>

#include "../../include/humanoid_env.h"

void hum_internal_set_error(const char* msg);

namespace {

constexpr int OBS = HUM_NOBS, ACT = HUM_NACT, H = 256, K1 = 72;   // K1: 70 padded to a multiple of 4
constexpr int ROWS = 16, WAVES = 4;

struct PolicyArgs {
    const float* w1; const float* b1; const float* w2; const float* b2; const float* w3; const float* b3;
    const float* log_std;
    const float* obs; const float* obs_reset; const unsigned char* done;
    float* act; float* mean_out; float* obs_in_out;
    int n, explore;
    unsigned long long seed, step;
};

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ inline unsigned long long mix64(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

// one 16 x (16 * NT) output slice of X[16 x K] (LDS, row stride ldx) times W[K x ncol] (global, row stride ldw):
// acc[t] = 16x16 tile t; lane l: A = X[l & 15][4s + (l >> 4)], B = W[4s + (l >> 4)][col0 + 16t + (l & 15)]
template <int NT>
__device__ inline void mfma_slice(const float* X, int ldx, int K, const float* __restrict__ W, int ldw, int col0,
                                  int ncol, f32x4* acc) {
    const int l = threadIdx.x & 63, r = l & 15, kq = l >> 4;
#pragma unroll
    for (int t = 0; t < NT; t++) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < K / 4; s++) {
        const int k = 4 * s + kq;
        const float a = X[r * ldx + k];
#pragma unroll
        for (int t = 0; t < NT; t++) {
            const int c = col0 + 16 * t + r;
            const float b = c < ncol ? W[(long)k * ldw + c] : 0.f;
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[t], 0, 0, 0);
        }
    }
}

__global__ void __launch_bounds__(64 * WAVES) policy_kernel(PolicyArgs p) {
    __shared__ float xs[ROWS][K1];
    __shared__ float h1[ROWS][H];
    __shared__ float h2[ROWS][H];
    const int tid = threadIdx.x, wave = tid >> 6, l = tid & 63;
    const int row0 = blockIdx.x * ROWS;
    // observation tile (done lanes read their post-reset observation: the sampler's next input)
    for (int e = tid; e < ROWS * K1; e += blockDim.x) {
        const int r = e / K1, k = e - r * K1, i = row0 + r;
        float v = 0.f;
        if (i < p.n && k < OBS) {
            const bool rs = p.obs_reset && p.done && p.done[i];
            v = (rs ? p.obs_reset : p.obs)[(long)i * OBS + k];
        }
        xs[r][k] = v;
        if (p.obs_in_out && i < p.n && k < OBS) p.obs_in_out[(long)i * OBS + k] = v;
    }
    __syncthreads();
    f32x4 acc[4];
    const int col0 = 64 * wave;
    // C/D map: lane l, register q -> row 4 (l >> 4) + q, column l & 15
    mfma_slice<4>(&xs[0][0], K1, K1, p.w1, H, col0, H, acc);
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = 4 * (l >> 4) + q, c = col0 + 16 * t + (l & 15);
            h1[r][c] = tanhf(acc[t][q] + p.b1[c]);
        }
    __syncthreads();
    mfma_slice<4>(&h1[0][0], H, H, p.w2, H, col0, H, acc);
#pragma unroll
    for (int t = 0; t < 4; t++)
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = 4 * (l >> 4) + q, c = col0 + 16 * t + (l & 15);
            h2[r][c] = tanhf(acc[t][q] + p.b2[c]);
        }
    __syncthreads();
    if (wave < 2) {   // output layer: 17 columns = two 16-wide tiles, one per wave
        f32x4 o[1];
        mfma_slice<1>(&h2[0][0], H, H, p.w3, ACT, 16 * wave, ACT, o);
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int r = 4 * (l >> 4) + q, c = 16 * wave + (l & 15), i = row0 + r;
            if (c < ACT && i < p.n) {
                const float mean = o[0][q] + p.b3[c];
                float a = mean;
                if (p.explore) {   // DiagGaussian sample: mean + exp(log_std) * N(0, 1), counter-based Box-Muller
                    const unsigned long long x = mix64(p.seed ^ mix64(((unsigned long long)i << 32) ^ (p.step * 32 + c)));
                    const float u1 = ((float)(x >> 40) + 1.f) * 0x1.0p-24f;   // (0, 1]
                    const float u2 = (float)((x >> 16) & 0xFFFFFFull) * 0x1.0p-24f;
                    a = mean + expf(p.log_std[c]) * sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
                }
                p.act[(long)i * ACT + c] = fminf(fmaxf(a, -1.f), 1.f);   // clip_actions (Box [-1, 1])
                if (p.mean_out) p.mean_out[(long)i * ACT + c] = mean;
            }
        }
    }
}

}  // namespace

struct hum_policy {
    int device;
    float* w;   // one allocation: w1 b1 w2 b2 w3 b3 log_std
    const float *w1, *b1, *w2, *b2, *w3, *b3, *log_std;
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
    if (!w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !out) return perr(HUM_ERR_ARG, "hum_policy_create: null argument");
    if (hipSetDevice(device) != hipSuccess) return perr(HUM_ERR_HIP, "hum_policy_create: hipSetDevice");
    // w1 is stored padded to K1 rows (rows 70, 71 zero) so the kernel's k loop needs no bound
    const size_t n1 = (size_t)K1 * H, n2 = (size_t)H * H, n3 = (size_t)H * ACT;
    const size_t total = n1 + H + n2 + H + n3 + ACT + ACT;
    hum_policy* p = new hum_policy();
    p->device = device;
    p->seed = seed;
    if (hipMalloc((void**)&p->w, total * sizeof(float)) != hipSuccess) {
        delete p;
        return perr(HUM_ERR_HIP, "hum_policy_create: hipMalloc");
    }
    float* h = new float[total]();
    std::memcpy(h, w1, (size_t)OBS * H * sizeof(float));
    size_t o = n1;
    std::memcpy(h + o, b1, H * sizeof(float)); o += H;
    std::memcpy(h + o, w2, n2 * sizeof(float)); o += n2;
    std::memcpy(h + o, b2, H * sizeof(float)); o += H;
    std::memcpy(h + o, w3, n3 * sizeof(float)); o += n3;
    std::memcpy(h + o, b3, ACT * sizeof(float)); o += ACT;
    if (log_std) std::memcpy(h + o, log_std, ACT * sizeof(float));
    const hipError_t st = hipMemcpy(p->w, h, total * sizeof(float), hipMemcpyHostToDevice);
    delete[] h;
    if (st != hipSuccess) {
        (void)hipFree(p->w);
        delete p;
        return perr(HUM_ERR_HIP, "hum_policy_create: hipMemcpy");
    }
    p->w1 = p->w; p->b1 = p->w1 + n1; p->w2 = p->b1 + H; p->b2 = p->w2 + n2; p->w3 = p->b2 + H;
    p->b3 = p->w3 + n3; p->log_std = p->b3 + ACT;
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
    if (!p || !obs || !actions || n <= 0) return perr(HUM_ERR_ARG, "hum_policy_act: bad argument");
    if ((obs_reset == nullptr) != (done == nullptr)) return perr(HUM_ERR_ARG, "hum_policy_act: obs_reset needs done");
    if (hipSetDevice(p->device) != hipSuccess) return perr(HUM_ERR_HIP, "hum_policy_act: hipSetDevice");
    PolicyArgs a;
    a.w1 = p->w1; a.b1 = p->b1; a.w2 = p->w2; a.b2 = p->b2; a.w3 = p->w3; a.b3 = p->b3; a.log_std = p->log_std;
    a.obs = obs; a.obs_reset = obs_reset; a.done = done; a.act = actions; a.mean_out = mean_out; a.obs_in_out = obs_in_out;
    a.n = n; a.explore = explore; a.seed = p->seed; a.step = step;
    hipLaunchKernelGGL(policy_kernel, dim3((n + ROWS - 1) / ROWS), dim3(64 * WAVES), 0, (hipStream_t)stream, a);
    const hipError_t st = hipGetLastError();
    if (st != hipSuccess) return perr(HUM_ERR_HIP, std::string("hum_policy_act: ") + hipGetErrorString(st));
    return HUM_OK;
}

// k sampler steps on the env's lanes with no host round trip: policy (on the current observation; lanes that
// finished an episode in the previous step act on their reset observation) -> hum_step with auto-reset.
// Trajectory outputs (device, any may be NULL): obs_traj [k,n,70] the policy's inputs, act_traj [k,n,17],
// rew_traj [k,n], done_traj [k,n].  obs / obs_reset / done / reward are the env-step buffers (device [n,70],
// [n,70], [n], [n]); on entry obs holds the current observation and done the previous step's flags (zeros after
// a reset).  Launches go to `stream` in order.
int hum_rollout(hum_env* env, hum_policy* p, int32_t k, int32_t explore, uint64_t step0, float* obs, float* obs_reset,
                uint8_t* done, float* reward, float* act_buf, float* obs_traj, float* act_traj, float* rew_traj,
                uint8_t* done_traj, void* stream) {
    if (!env || !p || k <= 0 || !obs || !obs_reset || !done || !reward || !act_buf)
        return perr(HUM_ERR_ARG, "hum_rollout: bad argument");
    const int n = hum_num_lanes(env);
    hipStream_t s = (hipStream_t)stream;
    for (int t = 0; t < k; t++) {
        int rc = hum_policy_act(p, obs, obs_reset, done, n, act_buf, nullptr,
                                obs_traj ? obs_traj + (size_t)t * n * HUM_NOBS : nullptr, explore, step0 + (uint64_t)t,
                                stream);
        if (rc != HUM_OK) return rc;
        rc = hum_step(env, act_buf, obs, reward, done, nullptr, HUM_STEP_AUTORESET, obs_reset, stream);
        if (rc != HUM_OK) return rc;
        if (act_traj && hipMemcpyAsync(act_traj + (size_t)t * n * HUM_NACT, act_buf, (size_t)n * HUM_NACT * sizeof(float),
                                       hipMemcpyDeviceToDevice, s) != hipSuccess)
            return perr(HUM_ERR_HIP, "hum_rollout: act copy");
        if (rew_traj && hipMemcpyAsync(rew_traj + (size_t)t * n, reward, (size_t)n * sizeof(float),
                                       hipMemcpyDeviceToDevice, s) != hipSuccess)
            return perr(HUM_ERR_HIP, "hum_rollout: reward copy");
        if (done_traj && hipMemcpyAsync(done_traj + (size_t)t * n, done, (size_t)n, hipMemcpyDeviceToDevice, s) != hipSuccess)
            return perr(HUM_ERR_HIP, "hum_rollout: done copy");
    }
    return HUM_OK;
}

}  // extern "C"
