// humanoid_env.hip - C-ABI (include/humanoid_env.h) of the vectorised humanoid env; device code in kernels.h.
//
// One launch = one env step for all lanes (4 physics substeps fused with the observation, imitation
// reward, frame/target bookkeeping and optional auto-reset).  One env per lane; lane state is SoA in
// HBM (element-major: value e of lane i at base[e * n + i]) so every load/store is coalesced.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "kernels.h"

using namespace hk;
using namespace hkk;

namespace {

thread_local std::string g_err;
int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
#define HIPCHK(x)                                                                              \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) return fail(HUM_ERR_HIP, std::string(#x ": ") + hipGetErrorString(e_)); \
    } while (0)

}  // namespace

// messages of host-side pieces in other translation units (clip_csv.cpp) go to hum_last_error() too
__attribute__((visibility("hidden"))) void hum_internal_set_error(const char* msg) { g_err = msg ? msg : ""; }


// ======================================================================================= C-ABI
struct hum_env {
    hum_config cfg;
    int n;
    hipStream_t stream;
    DevState d;
    size_t real_size;
    double* clip_dev[HUM_MAX_CLIPS];
    ClipDev clips[HUM_MAX_CLIPS];
    ClipDev* clips_dev;   // device copy of clips[] read by the kernels
    bool clip_set[HUM_MAX_CLIPS];
    double* pred;
    int npred;
    unsigned* eflags;
    // ground (hum_set_terrain)
    int terrain;
    float* hf;
    int hf_w, hf_l;
    double hf_s[3], hf_o[3], hf_mid;
    void* stage;          // HUM_STEP_HOST_IO: device staging for host buffers (grown on demand)
    size_t stage_bytes;
    void* traj;           // hum_rollout_fused without reward / done traces: their [k,n] rows (grown on demand)
    size_t traj_bytes;
    hipGraphExec_t graph;
    int graph_k;
    const void* graph_key[6];
    unsigned graph_flags;
};

namespace {
// block row pool capacity of the cooperative kernel: envs_per_block * MAXR_LDS LDS row slots, or fewer when
// hum_config.lds_rows asks (tests of the global spill path)
static int lds_rows_of(const hum_config& c) {
    const int pool = c.envs_per_block * MAXR_LDS;
    return c.lds_rows > 0 && c.lds_rows < pool ? c.lds_rows : pool;
}

KArgs make_args(hum_env* e) {
    KArgs a;
    memset(&a, 0, sizeof a);
    a.n = e->n;
    a.seed = e->cfg.seed;
    a.lane_offset = e->cfg.lane_offset;
    const hum_config& c = e->cfg;
    a.P.dt = c.dt_env / c.substeps;
    a.P.nsub = c.substeps;
    a.P.gravity = c.gravity;
    a.P.iters = c.solver_iters;
    a.P.erp_contact = c.erp_contact;
    a.P.erp_limit = c.erp_limit;
    a.P.split_pen = c.split_penetration;
    a.P.mu_ground = c.mu_ground;
    a.P.mu_self = c.mu_self;
    a.P.contact_thresh = c.contact_thresh;
    a.P.lin_damp = c.lin_damp;
    a.P.ang_damp = c.ang_damp;
    a.P.limit_max_impulse = c.limit_max_impulse;
    a.P.max_coord_vel = c.max_coord_vel;
    a.P.max_contacts = c.max_contacts;
    a.P.self_collision = c.self_collision;
    a.P.joint_damping = c.joint_damping;
    a.P.lds_rows = lds_rows_of(c);
    a.P.terrain = e->terrain;
    a.P.hf = e->hf;
    a.P.hf_w = e->hf_w;
    a.P.hf_l = e->hf_l;
    for (int k = 0; k < 3; k++) { a.P.hf_s[k] = e->hf_s[k]; a.P.hf_o[k] = e->hf_o[k]; }
    a.P.hf_mid = e->hf_mid;
    a.hier = c.hier;
    a.np1 = c.numpy_semantics == HUM_NUMPY_1;
    a.clips = e->clips_dev;
    a.pred = e->pred;
    a.npred = e->npred;
    a.phys = e->d.phys;
    a.bi = e->d.bi;
    a.bd = e->d.bd;
    a.scratch = e->d.scratch;
    a.eflags = e->eflags;
    a.ksteps = 1;
    return a;
}
dim3 grid_of(hum_env* e) { return dim3((e->n + e->cfg.block_size - 1) / e->cfg.block_size); }
hipStream_t stream_of(hum_env*, void* s) { return (hipStream_t)s; }   // NULL = HIP null stream
bool any_clip(hum_env* e) {
    for (int k = 0; k < HUM_MAX_CLIPS; k++)
        if (e->clip_set[k]) return true;
    return false;
}
}  // namespace

namespace {
int launch_step(hum_env* e, const KArgs& a, hipStream_t s);
// Inputs a captured step graph holds by value (clip descriptors, predefined course) are about to change:
// finish every launch that may read the old ones, then drop the graph so the next hum_step_graph recaptures.
hipError_t quiesce(hum_env* e) {
    hipError_t st = hipStreamSynchronize(e->stream);
    if (st == hipSuccess) st = hipDeviceSynchronize();   // launches on caller streams (hum_step(.., stream))
    if (e->graph) {
        (void)hipGraphExecDestroy(e->graph);
        e->graph = nullptr;
    }
    return st;
}
}  // namespace

extern "C" {

int hum_abi_version(void) { return HUM_ABI_VERSION; }
const char* hum_last_error(void) { return g_err.c_str(); }

void hum_default_config(hum_config* c) {
    memset(c, 0, sizeof *c);
    c->n_lanes = 1;
    c->device = 0;
    c->seed = 0;
    c->lane_offset = 0;
    c->precision = 0;
    c->block_size = 64;
    c->dt_env = 0.0165;
    c->substeps = 4;
    c->gravity = 9.8;
    c->solver_iters = 5;
    c->erp_contact = 0.9;
    c->erp_limit = 0.2;
    c->mu_ground = 2.0 * 0.8;
    c->mu_self = 2.0 * 2.0;
    c->contact_thresh = 0.02;
    c->lin_damp = 0.04;
    c->ang_damp = 0.04;
    c->limit_max_impulse = 100.0;
    c->max_coord_vel = 100.0;
    c->max_contacts = HUM_MAX_CONTACTS;   // every candidate: no truncation
    c->self_collision = 1;
    c->joint_damping = 1;
    c->kernel = 1;
    c->hier = 0;
    c->envs_per_block = 4;
    c->lds_rows = 0;
    c->numpy_semantics = HUM_NUMPY_1;
    c->split_penetration = -0.04;
}

int hum_create(const hum_config* cfg, hum_env** out) {
    if (!cfg || !out) return fail(HUM_ERR_ARG, "hum_create: null argument");
    if (cfg->n_lanes <= 0) return fail(HUM_ERR_ARG, "hum_create: n_lanes must be > 0");
    if (cfg->block_size <= 0 || cfg->block_size > 256 || cfg->block_size % 16)
        return fail(HUM_ERR_ARG, "hum_create: block_size must be a multiple of 16 in [16, 256]");
    if (cfg->precision != 0 && cfg->precision != 1) return fail(HUM_ERR_ARG, "hum_create: precision must be 0 or 1");
    if (cfg->substeps <= 0 || cfg->solver_iters < 0) return fail(HUM_ERR_ARG, "hum_create: bad solver settings");
    if (cfg->kernel != 0 && cfg->kernel != 1) return fail(HUM_ERR_ARG, "hum_create: kernel must be 0 (per-lane) or 1 (cooperative)");
    if (cfg->hier != 0 && cfg->hier != 1) return fail(HUM_ERR_ARG, "hum_create: hier must be 0 or 1");
    if (cfg->envs_per_block != 1 && cfg->envs_per_block != 2 && cfg->envs_per_block != 4)
        return fail(HUM_ERR_ARG, "hum_create: envs_per_block must be 1, 2 or 4");
    if (cfg->lds_rows < 0) return fail(HUM_ERR_ARG, "hum_create: lds_rows must be >= 0");
    if (cfg->numpy_semantics != HUM_NUMPY_1 && cfg->numpy_semantics != HUM_NUMPY_2)
        return fail(HUM_ERR_ARG, "hum_create: numpy_semantics must be HUM_NUMPY_1 or HUM_NUMPY_2");
    static_assert(MAXC_G == HUM_MAX_CONTACTS && MAXC == HUM_MAX_CONTACTS, "contact list holds every candidate");
    if (cfg->max_contacts < 0 || cfg->max_contacts > HUM_MAX_CONTACTS)
        return fail(HUM_ERR_ARG, "hum_create: max_contacts out of range [0, HUM_MAX_CONTACTS]");
    HIPCHK(hipSetDevice(cfg->device));
    hum_env* e = new hum_env();
    e->cfg = *cfg;
    e->n = cfg->n_lanes;
    e->real_size = cfg->precision ? sizeof(double) : sizeof(float);
    const size_t n = (size_t)e->n;
    hipError_t st = hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking);
    if (st == hipSuccess) st = hipMalloc(&e->d.phys, HUM_NSTATE * n * e->real_size);
    if (st == hipSuccess) st = hipMalloc((void**)&e->d.bi, NBOOK_I * n * sizeof(int));
    if (st == hipSuccess) st = hipMalloc((void**)&e->d.bd, NBOOK_D * n * sizeof(double));
    if (st == hipSuccess) {   // per-lane rows (kernel 0) or the per-block row spill regions (kernel 1)
        const int epb = cfg->envs_per_block;
        const size_t blocks = (n + epb - 1) / epb;
        st = hipMalloc(&e->d.scratch, (cfg->kernel == 1 ? (size_t)grow_block_size(epb, lds_rows_of(*cfg)) * blocks
                                                          : (size_t)SCRATCH_PER_LANE * n) * e->real_size);
    }
    if (st == hipSuccess) st = hipMalloc((void**)&e->eflags, sizeof(unsigned));
    if (st == hipSuccess) st = hipMalloc((void**)&e->clips_dev, HUM_MAX_CLIPS * sizeof(ClipDev));
    // zero-fill on the handle's own stream, so it is ordered before init_kernel: a plain hipMemset goes to the
    // null stream, which a non-blocking stream does not wait for, and a fill landing after init_kernel erased the
    // lanes' RNG keys (seen as an intermittent mismatch in test_gpu_multiproc)
    if (st == hipSuccess) st = hipMemsetAsync(e->clips_dev, 0, HUM_MAX_CLIPS * sizeof(ClipDev), e->stream);
    if (st == hipSuccess) st = hipMemsetAsync(e->d.bi, 0, NBOOK_I * n * sizeof(int), e->stream);
    if (st == hipSuccess) st = hipMemsetAsync(e->d.bd, 0, NBOOK_D * n * sizeof(double), e->stream);
    if (st == hipSuccess) st = hipMemsetAsync(e->d.phys, 0, HUM_NSTATE * n * e->real_size, e->stream);
    if (st == hipSuccess) st = hipMemsetAsync(e->eflags, 0, sizeof(unsigned), e->stream);
    if (st == hipSuccess) {
        KArgs a = make_args(e);
        hipLaunchKernelGGL(init_kernel, grid_of(e), dim3(e->cfg.block_size), 0, e->stream, a);
        st = hipGetLastError();
        if (st == hipSuccess) st = hipStreamSynchronize(e->stream);
    }
    if (st == hipSuccess && getenv("ILRL_DEBUG_PTRS")) {   // diagnostics: the device buffer map (fault addresses)
        const int epb = cfg->envs_per_block;
        const size_t sb = (cfg->kernel == 1 ? (size_t)grow_block_size(epb, lds_rows_of(*cfg)) * ((n + epb - 1) / epb)
                                            : (size_t)SCRATCH_PER_LANE * n) * e->real_size;
        fprintf(stderr, "hum_create %p: phys %p +%zu bi %p +%zu bd %p +%zu scratch %p +%zu eflags %p clips %p\n", (void*)e,
                e->d.phys, HUM_NSTATE * n * e->real_size, (void*)e->d.bi, NBOOK_I * n * sizeof(int), (void*)e->d.bd,
                NBOOK_D * n * sizeof(double), e->d.scratch, sb, (void*)e->eflags, (void*)e->clips_dev);
    }
    if (st != hipSuccess) {
        std::string m = std::string("hum_create: ") + hipGetErrorString(st);
        hum_destroy(e);
        return fail(HUM_ERR_HIP, m);
    }
    *out = e;
    return HUM_OK;
}

int hum_destroy(hum_env* e) {
    if (!e) return HUM_OK;
    (void)hipSetDevice(e->cfg.device);
    if (e->graph) (void)hipGraphExecDestroy(e->graph);
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    (void)hipFree(e->d.phys);
    (void)hipFree(e->d.bi);
    (void)hipFree(e->d.bd);
    (void)hipFree(e->d.scratch);
    (void)hipFree(e->eflags);
    (void)hipFree(e->clips_dev);
    (void)hipFree(e->pred);
    (void)hipFree(e->hf);
    (void)hipFree(e->stage);
    (void)hipFree(e->traj);
    for (int k = 0; k < HUM_MAX_CLIPS; k++) (void)hipFree(e->clip_dev[k]);
    if (e->stream) (void)hipStreamDestroy(e->stream);
    delete e;
    return HUM_OK;
}

int hum_set_clip(hum_env* e, int32_t id, const double* pos, int32_t n_pos, const double* vel, int32_t n_vel,
                 const double* rel, int32_t n_rel, const double* ep, int32_t n_ep) {
    if (!e || id < 0 || id >= HUM_MAX_CLIPS || !pos || !vel || !rel || !ep) return fail(HUM_ERR_ARG, "hum_set_clip: bad argument");
    if (n_pos < 8 || n_vel < 1 || n_rel < n_pos || n_ep < n_pos) return fail(HUM_ERR_ARG, "hum_set_clip: inconsistent table sizes");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(quiesce(e));
    if (e->clip_dev[id]) HIPCHK(hipFree(e->clip_dev[id]));
    const size_t np = (size_t)n_pos * 14, nv = (size_t)n_vel * 14, nr = (size_t)n_rel * 14, ne = (size_t)n_ep * 27;
    double* buf;
    HIPCHK(hipMalloc((void**)&buf, (np + nv + nr + ne) * sizeof(double)));
    HIPCHK(hipMemcpy(buf, pos, np * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(buf + np, vel, nv * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(buf + np + nv, rel, nr * sizeof(double), hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(buf + np + nv + nr, ep, ne * sizeof(double), hipMemcpyHostToDevice));
    e->clip_dev[id] = buf;
    if (getenv("ILRL_DEBUG_PTRS"))
        fprintf(stderr, "hum_set_clip %p: clip %d tables %p +%zu\n", (void*)e, id, (void*)buf, (np + nv + nr + ne) * sizeof(double));
    e->clips[id] = ClipDev{buf, buf + np, buf + np + nv, buf + np + nv + nr, n_pos, n_vel, n_rel, n_ep, n_pos - 1};
    e->clip_set[id] = true;
    HIPCHK(hipMemcpy(e->clips_dev + id, &e->clips[id], sizeof(ClipDev), hipMemcpyHostToDevice));
    return HUM_OK;
}

int hum_set_lane_clips(hum_env* e, const int32_t* clip_of_lane) {
    if (!e || !clip_of_lane) return fail(HUM_ERR_ARG, "hum_set_lane_clips: null argument");
    for (int i = 0; i < e->n; i++)
        if (clip_of_lane[i] < 0 || clip_of_lane[i] >= HUM_MAX_CLIPS || !e->clip_set[clip_of_lane[i]])
            return fail(HUM_ERR_NOCLIP, "hum_set_lane_clips: lane refers to a clip that was not uploaded");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(quiesce(e));   // in-flight launches (or graph replays) read the clip column
    HIPCHK(hipMemcpy(e->d.bi + 3 * e->n, clip_of_lane, e->n * sizeof(int), hipMemcpyHostToDevice));
    return HUM_OK;
}

int hum_set_lane_modes(hum_env* e, const uint32_t* modes) {
    if (!e || !modes) return fail(HUM_ERR_ARG, "hum_set_lane_modes: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(quiesce(e));
    HIPCHK(hipMemcpy(e->d.bi + 5 * e->n, modes, e->n * sizeof(int), hipMemcpyHostToDevice));
    return HUM_OK;
}

int hum_set_predefined_targets(hum_env* e, const double* xyz, int32_t n) {
    if (!e || (n > 0 && !xyz) || n < 0) return fail(HUM_ERR_ARG, "hum_set_predefined_targets: bad argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(quiesce(e));   // a captured graph holds pred / npred by value
    if (e->pred) HIPCHK(hipFree(e->pred));
    e->pred = nullptr;
    e->npred = n;
    if (n > 0) {
        HIPCHK(hipMalloc((void**)&e->pred, n * 3 * sizeof(double)));
        HIPCHK(hipMemcpy(e->pred, xyz, n * 3 * sizeof(double), hipMemcpyHostToDevice));
    }
    return HUM_OK;
}

int hum_set_terrain(hum_env* e, int32_t mode, const float* heights, int32_t w, int32_t l, const double* scale3,
                    const double* origin3) {
    return hum_set_terrain_ex(e, mode, heights, w, l, scale3, origin3, nullptr);
}

int hum_set_terrain_ex(hum_env* e, int32_t mode, const float* heights, int32_t w, int32_t l, const double* scale3,
                       const double* origin3, const double* centre) {
    if (!e) return fail(HUM_ERR_ARG, "hum_set_terrain: null env");
    if (mode != HUM_TERRAIN_PLANE && mode != HUM_TERRAIN_HEIGHTFIELD && mode != HUM_TERRAIN_RANDOM_BLOCKS)
        return fail(HUM_ERR_ARG, "hum_set_terrain: unknown mode");
    if (mode != HUM_TERRAIN_PLANE && (e->cfg.kernel != 1 || e->cfg.hier || e->cfg.envs_per_block != 4))
        return fail(HUM_ERR_STATE, "hum_set_terrain: terrain needs a low-level handle on the cooperative kernel "
                                   "(kernel 1, envs_per_block 4)");
    std::vector<float> h;
    double s[3] = {1, 1, 1}, o[3] = {0, 0, 0.25}, mid = 0.25;   // CustomScene: scale 1, body at z 0.25
    int W = 256, L = 256;
    if (mode == HUM_TERRAIN_HEIGHTFIELD) {
        if (!heights || !scale3 || !origin3 || w < 2 || l < 2) return fail(HUM_ERR_ARG, "hum_set_terrain: bad heightfield");
        if (!(scale3[0] >= 0.25 && scale3[1] >= 0.25 && scale3[2] > 0))
            return fail(HUM_ERR_ARG, "hum_set_terrain: scale x, y must be >= 0.25 and z > 0");
        W = w;
        L = l;
        h.assign(heights, heights + (size_t)w * l);
        float lo = h[0], hi = h[0];
        for (float v : h) {
            if (!std::isfinite(v)) return fail(HUM_ERR_ARG, "hum_set_terrain: non-finite height");
            lo = v < lo ? v : lo;
            hi = v > hi ? v : hi;
        }
        // btHeightfieldTerrainShape m_localOrigin: the (min + max) / 2 of the data the shape was CREATED with; a
        // replaceHeightfieldIndex update (CustomScene.replaceHeightfieldData) keeps the creation value (centre)
        mid = centre ? *centre : 0.5 * ((double)lo + (double)hi);
        if (!std::isfinite(mid)) return fail(HUM_ERR_ARG, "hum_set_terrain: non-finite centre");
        for (int k = 0; k < 3; k++) { s[k] = scale3[k]; o[k] = origin3[k]; }
    }
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(quiesce(e));   // launches in flight (and a captured graph) hold the old terrain by value
    if (e->hf) HIPCHK(hipFree(e->hf));
    e->hf = nullptr;
    if (mode == HUM_TERRAIN_HEIGHTFIELD) {
        HIPCHK(hipMalloc((void**)&e->hf, h.size() * sizeof(float)));
        HIPCHK(hipMemcpy(e->hf, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    e->terrain = mode;
    e->hf_w = W;
    e->hf_l = L;
    for (int k = 0; k < 3; k++) { e->hf_s[k] = s[k]; e->hf_o[k] = o[k]; }
    e->hf_mid = mid;
    return HUM_OK;
}

int hum_reset(hum_env* e, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
              float* obs_out, void* stream) {
    return hum_reset_ex(e, lane_mask, start_frame, reset_yaw_deg, 0u, obs_out, stream);
}

int hum_reset_ex(hum_env* e, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
                 uint32_t flags, float* obs_out, void* stream) {
    if (!e) return fail(HUM_ERR_ARG, "hum_reset: null env");
    if (flags & ~(HUM_RESET_NO_REF_POSE | HUM_RESET_NO_INIT_VEL)) return fail(HUM_ERR_ARG, "hum_reset: unknown flags");
    if (e->cfg.hier) return fail(HUM_ERR_STATE, "hum_reset: hierarchical handle (use hum_hier_reset)");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_reset: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.mask = lane_mask;
    a.start_frame = start_frame;
    a.reset_yaw = reset_yaw_deg;
    a.reset_flags = flags;
    a.obs = obs_out;
    hipStream_t s = stream_of(e, stream);
    if (e->cfg.precision) hipLaunchKernelGGL(reset_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    else hipLaunchKernelGGL(reset_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    HIPCHK(hipGetLastError());
    return HUM_OK;
}

}  // extern "C"

namespace {
// HUM_STEP_HOST_IO: the hot-path buffers are host pointers.  Stage them through one device allocation on the launch
// stream (inputs and outputs copied in - outputs too, so rows a step leaves unwritten keep the caller's values -, the
// launch, outputs copied back), then synchronise.  bufs[j].p points at the argument slot, rewritten to the staging
// address for the launch.
struct HostBuf { const void** p; size_t bytes; bool out; };
template <typename F>
int staged(hum_env* e, hipStream_t s, HostBuf* bufs, int nb, F launch) {
    size_t total = 0;
    for (int j = 0; j < nb; j++)
        if (*bufs[j].p) total += (bufs[j].bytes + 255) / 256 * 256;
    if (total > e->stage_bytes) {
        HIPCHK(hipStreamSynchronize(s));
        if (e->stage) HIPCHK(hipFree(e->stage));
        e->stage = nullptr;
        e->stage_bytes = 0;
        HIPCHK(hipMalloc(&e->stage, total));
        e->stage_bytes = total;
    }
    const void* host[16];
    size_t off = 0;
    for (int j = 0; j < nb; j++) {
        host[j] = *bufs[j].p;
        if (!host[j]) continue;
        void* d = (char*)e->stage + off;
        off += (bufs[j].bytes + 255) / 256 * 256;
        HIPCHK(hipMemcpyAsync(d, host[j], bufs[j].bytes, hipMemcpyHostToDevice, s));
        *bufs[j].p = d;
    }
    const int rc = launch();
    for (int j = 0; j < nb; j++) {
        if (host[j] && bufs[j].out && rc == HUM_OK)
            HIPCHK(hipMemcpyAsync(const_cast<void*>(host[j]), *bufs[j].p, bufs[j].bytes, hipMemcpyDeviceToHost, s));
        *bufs[j].p = host[j];
    }
    HIPCHK(hipStreamSynchronize(s));
    return rc;
}
// HUM_STEP_CHECK_FINITE, before the launch: take the non-finite-action bit out of the sticky flags on the stream, so
// that the check after the launch reports this call's actions only (an earlier unchecked asynchronous step may have
// left it set)
__global__ void clear_eflag_kernel(unsigned* eflags, unsigned bits) {
    if (threadIdx.x == 0) atomicAnd(eflags, ~bits);
}
int clear_nonfinite(hum_env* e, hipStream_t s) {
    hipLaunchKernelGGL(clear_eflag_kernel, dim3(1), dim3(64), 0, s, e->eflags, (unsigned)HUM_EFLAG_NONFINITE_ACTION);
    HIPCHK(hipGetLastError());
    return HUM_OK;
}
// HUM_STEP_CHECK_FINITE: wait for the launch and turn a non-finite action (humanoid.py:55 assert) into an error
// status; the bit is taken out of the sticky flags
int check_finite(hum_env* e, hipStream_t s) {
    unsigned v = 0;
    HIPCHK(hipMemcpyAsync(&v, e->eflags, sizeof v, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!(v & HUM_EFLAG_NONFINITE_ACTION)) return HUM_OK;
    const unsigned w = v & ~HUM_EFLAG_NONFINITE_ACTION;
    HIPCHK(hipMemcpyAsync(e->eflags, &w, sizeof w, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    return fail(HUM_ERR_ARG, "hum_step: non-finite action (humanoid.py:55 assert np.isfinite(a).all()): those lanes "
                             "were not stepped");
}
constexpr uint32_t STEP_FLAGS = HUM_STEP_AUTORESET | HUM_STEP_SKIP_PHYSICS | HUM_STEP_HOST_IO | HUM_STEP_CHECK_FINITE;
}  // namespace

extern "C" {

int hum_step(hum_env* e, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
             uint32_t flags, float* obs_reset, void* stream) {
    return hum_step_k(e, actions, obs, reward, done, frame, flags, obs_reset, 1, stream);
}

int hum_step_k(hum_env* e, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
               uint32_t flags, float* obs_reset, int32_t k, void* stream) {
    if (!e || !actions || !obs || !reward || !done) return fail(HUM_ERR_ARG, "hum_step: null argument");
    if (k < 1) return fail(HUM_ERR_ARG, "hum_step_k: k must be >= 1");
    if (flags & ~STEP_FLAGS) return fail(HUM_ERR_ARG, "hum_step: unknown flags");
    if (e->cfg.hier) return fail(HUM_ERR_STATE, "hum_step: hierarchical handle (use hum_hier_step)");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_step: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.act = actions;
    a.obs = obs;
    a.rew = reward;
    a.done = done;
    a.frame_out = frame;
    a.flags = flags & (HUM_STEP_AUTORESET | HUM_STEP_SKIP_PHYSICS);
    a.obs_reset = obs_reset;
    a.ksteps = k;
    const hipStream_t s = stream_of(e, stream);
    int rc;
    if ((flags & HUM_STEP_CHECK_FINITE) && (rc = clear_nonfinite(e, s)) != HUM_OK) return rc;
    if (flags & HUM_STEP_HOST_IO) {
        const size_t kn = (size_t)k * e->n;
        HostBuf b[6] = {{(const void**)&a.act, kn * HUM_NACT * 4, false}, {(const void**)&a.obs, kn * HUM_NOBS * 4, true},
                        {(const void**)&a.rew, kn * 4, true}, {(const void**)&a.done, kn, true},
                        {(const void**)&a.frame_out, kn * 4, true}, {(const void**)&a.obs_reset, kn * HUM_NOBS * 4, true}};
        rc = staged(e, s, b, 6, [&] { return launch_step(e, a, s); });
    } else {
        rc = launch_step(e, a, s);
    }
    if (rc == HUM_OK && (flags & HUM_STEP_CHECK_FINITE)) rc = check_finite(e, s);
    return rc;
}

int hum_hier_reset(hum_env* e, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
                   float* high_obs_out, void* stream) {
    return hum_hier_reset_ex(e, lane_mask, start_frame, reset_yaw_deg, 0u, high_obs_out, stream);
}

int hum_hier_reset_ex(hum_env* e, const uint8_t* lane_mask, const int32_t* start_frame, const double* reset_yaw_deg,
                      uint32_t flags, float* high_obs_out, void* stream) {
    if (!e) return fail(HUM_ERR_ARG, "hum_hier_reset: null env");
    if (flags & ~(HUM_RESET_NO_REF_POSE | HUM_RESET_NO_INIT_VEL)) return fail(HUM_ERR_ARG, "hum_hier_reset: unknown flags");
    if (!e->cfg.hier) return fail(HUM_ERR_STATE, "hum_hier_reset: handle was not created with hier = 1");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_hier_reset: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.mask = lane_mask;
    a.start_frame = start_frame;
    a.reset_yaw = reset_yaw_deg;
    a.reset_flags = flags;
    a.obs_high = high_obs_out;
    hipStream_t s = stream_of(e, stream);
    if (e->cfg.precision) hipLaunchKernelGGL(reset_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    else hipLaunchKernelGGL(reset_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    HIPCHK(hipGetLastError());
    return HUM_OK;
}

int hum_hier_step(hum_env* e, const float* high_act, const float* low_act, const uint8_t* agent, uint8_t* agents,
                  float* high_obs, float* low_obs, float* high_rew, float* low_rew, uint8_t* done, int32_t* frame,
                  uint32_t flags, float* high_obs_reset, void* stream) {
    return hum_hier_step_k(e, high_act, low_act, agent, agents, high_obs, low_obs, high_rew, low_rew, done, frame, flags,
                           high_obs_reset, 1, stream);
}

int hum_hier_step_k(hum_env* e, const float* high_act, const float* low_act, const uint8_t* agent, uint8_t* agents,
                    float* high_obs, float* low_obs, float* high_rew, float* low_rew, uint8_t* done, int32_t* frame,
                    uint32_t flags, float* high_obs_reset, int32_t k, void* stream) {
    if (!e || !high_act || !low_act || !agents || !high_obs || !low_obs || !high_rew || !low_rew || !done)
        return fail(HUM_ERR_ARG, "hum_hier_step: null argument");
    if (k < 1) return fail(HUM_ERR_ARG, "hum_hier_step_k: k must be >= 1");
    if (flags & ~STEP_FLAGS) return fail(HUM_ERR_ARG, "hum_hier_step: unknown flags");
    if (!e->cfg.hier) return fail(HUM_ERR_STATE, "hum_hier_step: handle was not created with hier = 1");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_hier_step: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.act = low_act;
    a.act_high = high_act;
    a.agent_sel = agent;
    a.agents = agents;
    a.obs = low_obs;
    a.obs_high = high_obs;
    a.rew = low_rew;
    a.rew_high = high_rew;
    a.done = done;
    a.frame_out = frame;
    a.flags = flags & (HUM_STEP_AUTORESET | HUM_STEP_SKIP_PHYSICS);
    a.obs_high_reset = high_obs_reset;
    a.ksteps = k;
    const hipStream_t s = stream_of(e, stream);
    int rc;
    if ((flags & HUM_STEP_CHECK_FINITE) && (rc = clear_nonfinite(e, s)) != HUM_OK) return rc;
    if (flags & HUM_STEP_HOST_IO) {
        const size_t kn = (size_t)k * e->n;
        HostBuf b[12] = {{(const void**)&a.act, kn * HUM_NACT * 4, false},
                         {(const void**)&a.act_high, kn * HUM_NACT_HIGH * 4, false},
                         {(const void**)&a.agent_sel, kn, false}, {(const void**)&a.agents, kn, true},
                         {(const void**)&a.obs_high, kn * HUM_NOBS_HIGH * 4, true},
                         {(const void**)&a.obs, kn * HUM_NOBS * 4, true}, {(const void**)&a.rew_high, kn * 4, true},
                         {(const void**)&a.rew, kn * 4, true}, {(const void**)&a.done, kn, true},
                         {(const void**)&a.frame_out, kn * 4, true},
                         {(const void**)&a.obs_high_reset, kn * HUM_NOBS_HIGH * 4, true}, {nullptr, 0, false}};
        rc = staged(e, s, b, 11, [&] { return launch_step(e, a, s); });
    } else {
        rc = launch_step(e, a, s);
    }
    if (rc == HUM_OK && (flags & HUM_STEP_CHECK_FINITE)) rc = check_finite(e, s);
    return rc;
}

}  // extern "C"

namespace {
int launch_step(hum_env* e, const KArgs& a, hipStream_t s) {
#ifdef HUM_DIAG_F32_ONLY   // diagnostic builds (phase timing): only the benchmarked kernel is instantiated
#ifndef HUM_DIAG_EPB
#define HUM_DIAG_EPB 4
#endif
    if (e->cfg.kernel != 1 || e->cfg.precision || e->cfg.envs_per_block != HUM_DIAG_EPB || e->terrain)
        return fail(HUM_ERR_ARG, "diagnostic build: only kernel 1, fp32, envs_per_block HUM_DIAG_EPB, plane");
    if (a.hier) hipLaunchKernelGGL((step_group_kernel<float, HUM_DIAG_EPB, false, 4>), dim3((e->n + HUM_DIAG_EPB - 1) / HUM_DIAG_EPB),
                                   dim3(HUM_DIAG_EPB * GL), 0, s, a);
    else hipLaunchKernelGGL((step_group_kernel<float, HUM_DIAG_EPB, false, 3>), dim3((e->n + HUM_DIAG_EPB - 1) / HUM_DIAG_EPB),
                            dim3(HUM_DIAG_EPB * GL), 0, s, a);
#else
    if (e->cfg.kernel == 1) {
        const int epb = e->cfg.envs_per_block;
        const dim3 g((e->n + epb - 1) / epb), blk(epb * GL);
        if (e->terrain != HUM_TERRAIN_PLANE) {   // heightfield ground: its own instantiation (envs_per_block 4)
            if (e->cfg.precision) hipLaunchKernelGGL((step_group_kernel<double, 4, true>), g, blk, 0, s, a);
            else hipLaunchKernelGGL((step_group_kernel<float, 4, true>), g, blk, 0, s, a);
        } else if (e->cfg.precision) {
            if (epb == 4) hipLaunchKernelGGL((step_group_kernel<double, 4>), g, blk, 0, s, a);
            else if (epb == 2) hipLaunchKernelGGL((step_group_kernel<double, 2>), g, blk, 0, s, a);
            else hipLaunchKernelGGL((step_group_kernel<double, 1>), g, blk, 0, s, a);
        } else {
            if (epb == 4) {
#ifdef HUM_SINGLE_TU
                if (a.hier) hipLaunchKernelGGL((step_group_kernel<float, 4, false, 4>), g, blk, 0, s, a);
                else hipLaunchKernelGGL((step_group_kernel<float, 4, false, 3>), g, blk, 0, s, a);
#else
                if (a.hier) HIPCHK(launch_group_f32_4(a, (int)g.x, s));
                else HIPCHK(launch_group_f32_4_low(a, (int)g.x, s));   // the benchmarked kernel
#endif
            }
            else if (epb == 2) hipLaunchKernelGGL((step_group_kernel<float, 2>), g, blk, 0, s, a);
            else hipLaunchKernelGGL((step_group_kernel<float, 1>), g, blk, 0, s, a);
        }
    } else {
        if (e->cfg.precision) hipLaunchKernelGGL(step_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
        else hipLaunchKernelGGL(step_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    }
#endif
    HIPCHK(hipGetLastError());
    return HUM_OK;
}
}  // namespace

extern "C" {

int hum_step_graph(hum_env* e, const float* actions, float* obs, float* reward, uint8_t* done, int32_t* frame,
                   uint32_t flags, float* obs_reset, int32_t k) {
    if (!e || k <= 0) return fail(HUM_ERR_ARG, "hum_step_graph: bad argument");
    if (flags & (HUM_STEP_HOST_IO | HUM_STEP_CHECK_FINITE))
        return fail(HUM_ERR_ARG, "hum_step_graph: HUM_STEP_HOST_IO / HUM_STEP_CHECK_FINITE synchronise (not capturable)");
    HIPCHK(hipSetDevice(e->cfg.device));
    const void* key[6] = {actions, obs, reward, done, frame, obs_reset};
    bool same = e->graph && e->graph_k == k && e->graph_flags == flags && memcmp(key, e->graph_key, sizeof key) == 0;
    if (!same) {
        if (e->graph) { (void)hipGraphExecDestroy(e->graph); e->graph = nullptr; }
        hipGraph_t g;
        HIPCHK(hipStreamBeginCapture(e->stream, hipStreamCaptureModeThreadLocal));
        for (int t = 0; t < k; t++) {
            int r = hum_step(e, actions, obs, reward, done, frame, flags, obs_reset, e->stream);
            if (r != HUM_OK) {
                (void)hipStreamEndCapture(e->stream, &g);
                return r;
            }
        }
        HIPCHK(hipStreamEndCapture(e->stream, &g));
        HIPCHK(hipGraphInstantiate(&e->graph, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
        e->graph_k = k;
        e->graph_flags = flags;
        memcpy(e->graph_key, key, sizeof key);
    }
    HIPCHK(hipGraphLaunch(e->graph, e->stream));
    return HUM_OK;
}

int hum_get_aux(hum_env* e, float* aux_out, void* stream) {
    if (!e || !aux_out) return fail(HUM_ERR_ARG, "hum_get_aux: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.aux = aux_out;
    hipStream_t s = stream_of(e, stream);
    if (e->cfg.precision) hipLaunchKernelGGL(aux_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    else hipLaunchKernelGGL(aux_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, s, a);
    HIPCHK(hipGetLastError());
    return HUM_OK;
}

int hum_get_state(hum_env* e, double* phys, double* book) {
    if (!e) return fail(HUM_ERR_ARG, "hum_get_state: null env");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    const size_t n = e->n;
    if (phys) {
        std::vector<unsigned char> tmp(HUM_NSTATE * n * e->real_size);
        HIPCHK(hipMemcpy(tmp.data(), e->d.phys, tmp.size(), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++)
            for (int k = 0; k < HUM_NSTATE; k++)
                phys[i * HUM_NSTATE + k] = e->cfg.precision ? ((double*)tmp.data())[k * n + i] : (double)((float*)tmp.data())[k * n + i];
    }
    if (book) {
        std::vector<int> bi(NBOOK_I * n);
        std::vector<double> bd(NBOOK_D * n);
        HIPCHK(hipMemcpy(bi.data(), e->d.bi, bi.size() * sizeof(int), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(bd.data(), e->d.bd, bd.size() * sizeof(double), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n; i++) {
            double* o = book + i * HUM_NBOOK;
            memset(o, 0, HUM_NBOOK * sizeof(double));
            o[HUM_BK_FRAME] = bi[0 * n + i];
            o[HUM_BK_TIMESTEP] = bi[1 * n + i];
            o[HUM_BK_PRED_INDEX] = bi[2 * n + i];
            o[HUM_BK_CLIP] = bi[3 * n + i];
            o[HUM_BK_RNG_COUNTER] = (double)(unsigned)bi[4 * n + i];
            o[HUM_BK_MODE] = (double)(unsigned)bi[5 * n + i];
            o[HUM_BK_RNG_KEY_LO] = (double)(unsigned)bi[6 * n + i];
            o[HUM_BK_RNG_KEY_HI] = (double)(unsigned)bi[7 * n + i];
            for (int k = 0; k < 3; k++) {
                o[HUM_BK_TARGET + k] = bd[(0 + k) * n + i];
                o[HUM_BK_START_ROBOT_POS + k] = bd[(3 + k) * n + i];
                o[HUM_BK_ROBOT_POS + k] = bd[(6 + k) * n + i];
                o[HUM_BK_START_EP_POS + k] = bd[(9 + k) * n + i];
            }
            o[HUM_BK_HL_DEG_TARGET] = bd[12 * n + i];
            o[HUM_BK_WALK_TARGET] = bd[13 * n + i];
            o[HUM_BK_WALK_TARGET + 1] = bd[14 * n + i];
            o[HUM_BK_LOW_TARGET_SCORE] = bd[15 * n + i];
            o[HUM_BK_DELTA_JOINTS] = bd[16 * n + i];
            o[HUM_BK_DELTA_VEL_JOINTS] = bd[17 * n + i];
            o[HUM_BK_BODY_POSTURE] = bd[18 * n + i];
            o[HUM_BK_ELECTRICITY] = bd[19 * n + i];
            o[HUM_BK_JOINT_LIMIT] = bd[20 * n + i];
            o[HUM_BK_ALIVE] = bd[21 * n + i];
            o[HUM_BK_DELTA_LOW_TARGET] = bd[22 * n + i];
            o[HUM_BK_LEVEL_REMAINING] = bi[8 * n + i];
            o[HUM_BK_NUM_HIGH_STEPS] = bi[9 * n + i];
            o[HUM_BK_EXPECT_HIGH] = bi[10 * n + i];
            o[HUM_BK_HIGH_TARGET_SCORE] = bd[23 * n + i];
            o[HUM_BK_CUM_DRIFT] = bd[24 * n + i];
            o[HUM_BK_DRIFT] = bd[25 * n + i];
            o[HUM_BK_DELTA_HIGH_TARGET] = bd[26 * n + i];
            o[HUM_BK_CUM_ALIVE] = bd[27 * n + i];
            o[HUM_BK_BODY_XY] = bd[28 * n + i];
            o[HUM_BK_BODY_XY + 1] = bd[29 * n + i];
            o[HUM_BK_TERRAIN_KEY_LO] = (double)(unsigned)bi[11 * n + i];
            o[HUM_BK_TERRAIN_KEY_HI] = (double)(unsigned)bi[12 * n + i];
        }
    }
    return HUM_OK;
}

int hum_set_state(hum_env* e, const double* phys, const double* book) {
    if (!e) return fail(HUM_ERR_ARG, "hum_set_state: null env");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    const size_t n = e->n;
    if (phys) {
        std::vector<unsigned char> tmp(HUM_NSTATE * n * e->real_size);
        for (size_t i = 0; i < n; i++)
            for (int k = 0; k < HUM_NSTATE; k++) {
                if (e->cfg.precision) ((double*)tmp.data())[k * n + i] = phys[i * HUM_NSTATE + k];
                else ((float*)tmp.data())[k * n + i] = (float)phys[i * HUM_NSTATE + k];
            }
        HIPCHK(hipMemcpy(e->d.phys, tmp.data(), tmp.size(), hipMemcpyHostToDevice));
    }
    if (book) {
        std::vector<int> bi(NBOOK_I * n);
        std::vector<double> bd(NBOOK_D * n);
        for (size_t i = 0; i < n; i++) {
            const double* o = book + i * HUM_NBOOK;
            const int clip = (int)o[HUM_BK_CLIP];
            if (clip < 0 || clip >= HUM_MAX_CLIPS || !e->clip_set[clip])
                return fail(HUM_ERR_NOCLIP, "hum_set_state: lane clip id not uploaded");
            bi[0 * n + i] = (int)o[HUM_BK_FRAME];
            bi[1 * n + i] = (int)o[HUM_BK_TIMESTEP];
            bi[2 * n + i] = (int)o[HUM_BK_PRED_INDEX];
            bi[3 * n + i] = clip;
            bi[4 * n + i] = (int)(unsigned)o[HUM_BK_RNG_COUNTER];
            bi[5 * n + i] = (int)(unsigned)o[HUM_BK_MODE];
            bi[6 * n + i] = (int)(unsigned)o[HUM_BK_RNG_KEY_LO];
            bi[7 * n + i] = (int)(unsigned)o[HUM_BK_RNG_KEY_HI];
            for (int k = 0; k < 3; k++) {
                bd[(0 + k) * n + i] = o[HUM_BK_TARGET + k];
                bd[(3 + k) * n + i] = o[HUM_BK_START_ROBOT_POS + k];
                bd[(6 + k) * n + i] = o[HUM_BK_ROBOT_POS + k];
                bd[(9 + k) * n + i] = o[HUM_BK_START_EP_POS + k];
            }
            bd[12 * n + i] = o[HUM_BK_HL_DEG_TARGET];
            bd[13 * n + i] = o[HUM_BK_WALK_TARGET];
            bd[14 * n + i] = o[HUM_BK_WALK_TARGET + 1];
            bd[15 * n + i] = o[HUM_BK_LOW_TARGET_SCORE];
            bd[16 * n + i] = o[HUM_BK_DELTA_JOINTS];
            bd[17 * n + i] = o[HUM_BK_DELTA_VEL_JOINTS];
            bd[18 * n + i] = o[HUM_BK_BODY_POSTURE];
            bd[19 * n + i] = o[HUM_BK_ELECTRICITY];
            bd[20 * n + i] = o[HUM_BK_JOINT_LIMIT];
            bd[21 * n + i] = o[HUM_BK_ALIVE];
            bd[22 * n + i] = o[HUM_BK_DELTA_LOW_TARGET];
            bi[8 * n + i] = (int)o[HUM_BK_LEVEL_REMAINING];
            bi[9 * n + i] = (int)o[HUM_BK_NUM_HIGH_STEPS];
            bi[10 * n + i] = (int)o[HUM_BK_EXPECT_HIGH];
            bd[23 * n + i] = o[HUM_BK_HIGH_TARGET_SCORE];
            bd[24 * n + i] = o[HUM_BK_CUM_DRIFT];
            bd[25 * n + i] = o[HUM_BK_DRIFT];
            bd[26 * n + i] = o[HUM_BK_DELTA_HIGH_TARGET];
            bd[27 * n + i] = o[HUM_BK_CUM_ALIVE];
            bd[28 * n + i] = o[HUM_BK_BODY_XY];
            bd[29 * n + i] = o[HUM_BK_BODY_XY + 1];
            bi[11 * n + i] = (int)(unsigned)o[HUM_BK_TERRAIN_KEY_LO];
            bi[12 * n + i] = (int)(unsigned)o[HUM_BK_TERRAIN_KEY_HI];
        }
        HIPCHK(hipMemcpy(e->d.bi, bi.data(), bi.size() * sizeof(int), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(e->d.bd, bd.data(), bd.size() * sizeof(double), hipMemcpyHostToDevice));
    }
    return HUM_OK;
}

int hum_get_parts(hum_env* e, double* parts) {
    if (!e || !parts) return fail(HUM_ERR_ARG, "hum_get_parts: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    double* d;
    const size_t bytes = (size_t)e->n * NPART * 3 * sizeof(double);
    HIPCHK(hipMalloc((void**)&d, bytes));
    KArgs a = make_args(e);
    HIPCHK(hipDeviceSynchronize());
    if (e->cfg.precision) hipLaunchKernelGGL(parts_kernel<double>, grid_of(e), dim3(e->cfg.block_size), 0, e->stream, a, d);
    else hipLaunchKernelGGL(parts_kernel<float>, grid_of(e), dim3(e->cfg.block_size), 0, e->stream, a, d);
    hipError_t st = hipGetLastError();
    if (st == hipSuccess) st = hipDeviceSynchronize();
    if (st == hipSuccess) st = hipMemcpy(parts, d, bytes, hipMemcpyDeviceToHost);
    (void)hipFree(d);
    if (st != hipSuccess) return fail(HUM_ERR_HIP, std::string("hum_get_parts: ") + hipGetErrorString(st));
    return HUM_OK;
}

int hum_get_error_flags(hum_env* e, uint32_t* flags) {
    if (!e || !flags) return fail(HUM_ERR_ARG, "hum_get_error_flags: null argument");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    unsigned v = 0;
    HIPCHK(hipMemcpy(&v, e->eflags, sizeof v, hipMemcpyDeviceToHost));
    HIPCHK(hipMemsetAsync(e->eflags, 0, sizeof v, e->stream));   // done before any later launch (see hum_create)
    HIPCHK(hipStreamSynchronize(e->stream));
    *flags = v;
    return HUM_OK;
}

int hum_sync(hum_env* e) {
    if (!e) return fail(HUM_ERR_ARG, "hum_sync: null env");
    HIPCHK(hipSetDevice(e->cfg.device));
    HIPCHK(hipDeviceSynchronize());
    return HUM_OK;
}

int32_t hum_num_lanes(const hum_env* e) { return e ? e->n : 0; }

}  // extern "C"
__attribute__((visibility("hidden"))) int hum_internal_device(const hum_env* e) { return e ? e->cfg.device : -1; }
// hum_rollout_fused (policy.hip): k sampler steps in one launch of the fused-policy cooperative kernel.  pw: the
// hum_policy weight block.  Missing rew / done traces go to the handle's scratch (grown on demand, stream-ordered).
__attribute__((visibility("hidden"))) int hum_internal_rollout_fused(
    hum_env* e, const float* pw, uint64_t seed, int32_t k, int32_t explore, uint64_t step0, float* obs, float* obs_reset,
    uint8_t* done, float* reward, float* act_last, float* obs_traj, float* act_traj, float* rew_traj, uint8_t* done_traj,
    float* mean_traj, void* stream) {
    if (e->cfg.kernel != 1 || e->cfg.precision || e->cfg.envs_per_block != 4 || e->terrain != HUM_TERRAIN_PLANE ||
        e->cfg.hier)
        return fail(HUM_ERR_STATE, "hum_rollout_fused: needs the cooperative fp32 kernel, 4 envs per block, plane ground "
                                   "and the low-level env (use hum_rollout)");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_rollout_fused: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    const hipStream_t s = stream_of(e, stream);
    const size_t kn = (size_t)k * e->n;
    float* rt = rew_traj;
    uint8_t* dt = done_traj;
    if (!rt || !dt) {
        const size_t rbytes = (kn * sizeof(float) + 255) / 256 * 256, need = rbytes + kn;
        if (need > e->traj_bytes) {   // the previous launches using it are ordered before the free on this stream
            HIPCHK(hipStreamSynchronize(s));
            if (e->traj) HIPCHK(hipFree(e->traj));
            e->traj = nullptr;
            e->traj_bytes = 0;
            HIPCHK(hipMalloc(&e->traj, need));
            e->traj_bytes = need;
        }
        if (!rt) rt = (float*)e->traj;
        if (!dt) dt = (uint8_t*)e->traj + rbytes;
    }
    KArgs a = make_args(e);
    a.flags = HUM_STEP_AUTORESET;
    a.ksteps = k;
    a.obs = obs;
    a.obs_reset = obs_reset;
    a.done_in = done;
    a.rew = rt;
    a.done = dt;
    a.frame_out = nullptr;
    a.act = nullptr;
    a.pw = pw;
    a.pseed = seed;
    a.pstep0 = step0;
    a.pexplore = explore;
    a.obs_traj = obs_traj;
    a.act_traj = act_traj;
    a.act_last = act_last;
    a.mean_traj = mean_traj;
    const int nb = (e->n + 3) / 4;
#ifndef HUM_DIAG_F32_ONLY
    hipError_t st = launch_group_f32_4_policy(a, nb, s);
#else   // diagnostic builds link the benchmarked kernel's phase-timed copy only
    (void)nb;
    hipError_t st = hipErrorInvalidDeviceFunction;
#endif
    if (st == hipSuccess) st = hipMemcpyAsync(reward, rt + (k - 1) * (size_t)e->n, (size_t)e->n * sizeof(float),
                                              hipMemcpyDeviceToDevice, s);
    if (st == hipSuccess) st = hipMemcpyAsync(done, dt + (k - 1) * (size_t)e->n, (size_t)e->n, hipMemcpyDeviceToDevice, s);
    if (st != hipSuccess) return fail(HUM_ERR_HIP, std::string("hum_rollout_fused: ") + hipGetErrorString(st));
    return HUM_OK;
}
// hum_hier_rollout_fused (policy.hip): k two-level sampler transitions in one launch of the cooperative kernel with
// both networks inside (POLICY == 2).  pw_high / pw_low: the hum_policy weight blocks.  The per-transition agents /
// rewards / done rows go to the trajectory when given, else to the handle's scratch (grown on demand,
// stream-ordered: every call on one handle must use one stream, or order its streams with events)
__attribute__((visibility("hidden"))) int hum_internal_hier_rollout_fused(
    hum_env* e, const float* pw_high, uint64_t seed_high, const float* pw_low, uint64_t seed_low, int32_t k,
    int32_t explore, uint64_t step0, const hum_hier_io* io, const hum_hier_traj* T, float* mean_high, float* mean_low,
    void* stream) {
    if (e->cfg.kernel != 1 || e->cfg.precision || e->cfg.envs_per_block != 4 || e->terrain != HUM_TERRAIN_PLANE ||
        !e->cfg.hier)
        return fail(HUM_ERR_STATE, "hum_hier_rollout_fused: needs a hierarchical handle on the cooperative fp32 kernel, "
                                   "4 envs per block and plane ground (use hum_hier_rollout)");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_hier_rollout_fused: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    const hipStream_t s = stream_of(e, stream);
    const size_t n = (size_t)e->n, kn = (size_t)k * n;
    float* rh = T->rew_high;
    float* rl = T->rew_low;
    uint8_t* ag = T->agents;
    uint8_t* dn = T->done;
    if (!rh || !rl || !ag || !dn) {
        const size_t fb = (kn * sizeof(float) + 255) / 256 * 256, bb = (kn + 255) / 256 * 256, need = 2 * fb + 2 * bb;
        if (need > e->traj_bytes) {   // the previous launches using it are ordered before the free on this stream
            HIPCHK(hipStreamSynchronize(s));
            if (e->traj) HIPCHK(hipFree(e->traj));
            e->traj = nullptr;
            e->traj_bytes = 0;
            HIPCHK(hipMalloc(&e->traj, need));
            e->traj_bytes = need;
        }
        char* base = (char*)e->traj;
        if (!rh) rh = (float*)base;
        if (!rl) rl = (float*)(base + fb);
        if (!ag) ag = (uint8_t*)(base + 2 * fb);
        if (!dn) dn = (uint8_t*)(base + 2 * fb + bb);
    }
    KArgs a = make_args(e);
    a.flags = HUM_STEP_AUTORESET;
    a.ksteps = k;
    a.obs = io->obs_low;
    a.obs_high = io->obs_high;
    a.obs_high_reset = io->obs_high_reset;
    a.done_in = io->done;
    a.rew = rl;
    a.rew_high = rh;
    a.agents = ag;
    a.done = dn;
    a.acted = T->acted;
    a.pw = pw_low;
    a.pseed = seed_low;
    a.obs_traj = T->obs_low;
    a.act_traj = T->act_low;
    a.act_last = io->act_low;
    a.pw_high = pw_high;
    a.pseed_high = seed_high;
    a.obs_traj_high = T->obs_high;
    a.act_traj_high = T->act_high;
    a.act_last_high = io->act_high;
    a.mean_traj = mean_low;
    a.mean_traj_high = mean_high;
    a.pstep0 = step0;
    a.pexplore = explore;
    const int nb = (e->n + 3) / 4;
#ifndef HUM_DIAG_F32_ONLY
    hipError_t st = launch_group_f32_4_hier_policy(a, nb, s);
#else
    (void)nb;
    hipError_t st = hipErrorInvalidDeviceFunction;
#endif
    // the last transition's rows into the env buffers
    const size_t last = (size_t)(k - 1) * n;
    if (st == hipSuccess) st = hipMemcpyAsync(io->agents, ag + last, n, hipMemcpyDeviceToDevice, s);
    if (st == hipSuccess) st = hipMemcpyAsync(io->rew_high, rh + last, n * sizeof(float), hipMemcpyDeviceToDevice, s);
    if (st == hipSuccess) st = hipMemcpyAsync(io->rew_low, rl + last, n * sizeof(float), hipMemcpyDeviceToDevice, s);
    if (st == hipSuccess) st = hipMemcpyAsync(io->done, dn + last, n, hipMemcpyDeviceToDevice, s);
    if (st != hipSuccess) return fail(HUM_ERR_HIP, std::string("hum_hier_rollout_fused: ") + hipGetErrorString(st));
    return HUM_OK;
}
// one hierarchical transition (hum_hier_step, agent = each lane's expected one) that also records the agent that
// acted per lane (acted [n], may be NULL): hum_hier_rollout's env launch (policy.hip)
__attribute__((visibility("hidden"))) int hum_internal_hier_step_acted(
    hum_env* e, const float* high_act, const float* low_act, uint8_t* agents, float* high_obs, float* low_obs,
    float* high_rew, float* low_rew, uint8_t* done, uint32_t flags, float* high_obs_reset, uint8_t* acted,
    void* stream) {
    if (!e || !high_act || !low_act || !agents || !high_obs || !low_obs || !high_rew || !low_rew || !done)
        return fail(HUM_ERR_ARG, "hum_hier_rollout: null argument");
    if (!e->cfg.hier) return fail(HUM_ERR_STATE, "hum_hier_rollout: handle was not created with hier = 1");
    if (!any_clip(e)) return fail(HUM_ERR_NOCLIP, "hum_hier_rollout: no clip uploaded (hum_set_clip)");
    HIPCHK(hipSetDevice(e->cfg.device));
    KArgs a = make_args(e);
    a.act = low_act;
    a.act_high = high_act;
    a.agents = agents;
    a.obs = low_obs;
    a.obs_high = high_obs;
    a.rew = low_rew;
    a.rew_high = high_rew;
    a.done = done;
    a.flags = flags & (HUM_STEP_AUTORESET | HUM_STEP_SKIP_PHYSICS);
    a.obs_high_reset = high_obs_reset;
    a.acted = acted;
    a.ksteps = 1;
    return launch_step(e, a, stream_of(e, stream));
}
extern "C" {


#ifdef HUM_WLOG_ON
int hum_debug_wave_log(unsigned* out, int nblocks, int reset) {   // diag: per-block work log (WLOG_W u32 each)
    HIPCHK(hipDeviceSynchronize());
    if (nblocks > 65536) nblocks = 65536;
    if (out) HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_log), (size_t)nblocks * WLOG_W * sizeof(unsigned)));
    if (reset) {
        void* p = nullptr;
        HIPCHK(hipGetSymbolAddress(&p, HIP_SYMBOL(g_wave_log)));
        HIPCHK(hipMemset(p, 0, sizeof(g_wave_log)));
    }
    return HUM_OK;
}
#endif

#ifdef HUM_PHASE_TIMING
// diagnostic builds only: accumulated s_memtime cycles per cooperative-kernel phase (thread 0 of each block)
int hum_debug_phase_cycles(unsigned long long* out32, int reset) {
    HIPCHK(hipDeviceSynchronize());
    HIPCHK(hipMemcpyFromSymbol(out32, HIP_SYMBOL(g_phase_cycles), 32 * sizeof(unsigned long long)));
    if (reset) {
        unsigned long long z[32] = {0};
        HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_cycles), z, sizeof z));
    }
    return HUM_OK;
}
#endif
void* hum_stream(hum_env* e) { return e ? (void*)e->stream : nullptr; }

}  // extern "C"
