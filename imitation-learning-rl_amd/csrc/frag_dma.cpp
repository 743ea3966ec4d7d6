// frag_dma.cpp - the learner feed's transport without compute units (include/humanoid_env.h hum_ipc_* / hum_dma_*).
//
// Why: the env kernel holds a whole SIMD register file per wave and four 40.8 KB blocks fill a CU's LDS, so while a
// hum_step_k launch runs no other kernel's wave is resident anywhere - an RCCL send / recv kernel (or a blit copy)
// waits for the launch to end, and config 4's gather (rank 0 pulls 7 x 46 MB per 32-step fragment) would serialise
// with the stepping.  The SDMA copy engines need no CU: each rank exports its packed send buffers once (IPC), and
// rank 0 pulls every peer's fragment with hsa_amd_memory_async_copy_on_engine forced onto an SDMA engine, over
// xGMI between GPUs (tools/micro/overlap.py: an SDMA transfer beside a running env launch is ~76 % hidden, a blit
// copy or a kernel on another stream waits for the launch).
//
// Host code only (HIP runtime for IPC, the HSA runtime for the copy engines); ordering against the producing and
// consuming streams is the caller's (ilrl_amd/parallel.py DmaGather: events + a host control channel).
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstring>
#include <mutex>
#include <string>

#include "../../include/humanoid_env.h"

void hum_internal_set_error(const char* msg);

namespace {

int fail(int code, const std::string& msg) {
    hum_internal_set_error(msg.c_str());
    return code;
}

std::once_flag g_hsa_once;
hsa_status_t g_hsa_init = HSA_STATUS_ERROR;

bool owner_agent(const void* p, hsa_agent_t* a) {
    hsa_amd_pointer_info_t pi;
    std::memset(&pi, 0, sizeof(pi));
    pi.size = sizeof(pi);
    if (hsa_amd_pointer_info(const_cast<void*>(p), &pi, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return false;
    if (pi.type == HSA_EXT_POINTER_TYPE_UNKNOWN) return false;
    *a = pi.agentOwner;
    return true;
}

}  // namespace

extern "C" int hum_ipc_export(const void* dev_ptr, uint8_t* handle, uint64_t* offset) {
    if (!dev_ptr || !handle || !offset) return fail(HUM_ERR_ARG, "hum_ipc_export: null argument");
    static_assert(sizeof(hipIpcMemHandle_t) <= HUM_IPC_HANDLE_BYTES, "IPC handle size");
    hipDeviceptr_t base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)dev_ptr) != hipSuccess)
        return fail(HUM_ERR_HIP, "hum_ipc_export: not a device allocation");
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, (void*)base);
    if (e != hipSuccess) return fail(HUM_ERR_HIP, std::string("hum_ipc_export: ") + hipGetErrorString(e));
    std::memset(handle, 0, HUM_IPC_HANDLE_BYTES);
    std::memcpy(handle, &h, sizeof(h));
    *offset = (uint64_t)((const char*)dev_ptr - (const char*)base);
    return HUM_OK;
}

extern "C" int hum_ipc_open(const uint8_t* handle, uint64_t offset, void** dev_ptr) {
    if (!handle || !dev_ptr) return fail(HUM_ERR_ARG, "hum_ipc_open: null argument");
    hipIpcMemHandle_t h;
    std::memcpy(&h, handle, sizeof(h));
    void* base = nullptr;
    const hipError_t e = hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return fail(HUM_ERR_HIP, std::string("hum_ipc_open: ") + hipGetErrorString(e));
    *dev_ptr = (char*)base + offset;
    return HUM_OK;
}

extern "C" int hum_ipc_close(void* base) {
    const hipError_t e = hipIpcCloseMemHandle(base);
    if (e != hipSuccess) return fail(HUM_ERR_HIP, std::string("hum_ipc_close: ") + hipGetErrorString(e));
    return HUM_OK;
}

extern "C" int hum_dma_copy(void* dst, const void* src, uint64_t bytes, int32_t engine, hum_dma_ticket* ticket) {
    if (!dst || !src || !ticket || engine < 0) return fail(HUM_ERR_ARG, "hum_dma_copy: bad argument");
    std::call_once(g_hsa_once, [] { g_hsa_init = hsa_init(); });   // reference-counted; HIP holds the runtime too
    if (g_hsa_init != HSA_STATUS_SUCCESS) return fail(HUM_ERR_HIP, "hum_dma_copy: hsa_init failed");
    hsa_agent_t da, sa;
    if (!owner_agent(dst, &da) || !owner_agent(src, &sa))
        return fail(HUM_ERR_ARG, "hum_dma_copy: dst / src is not memory of a GPU agent");
    hsa_signal_t sig;
    if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return fail(HUM_ERR_HIP, "hum_dma_copy: signal");
    // the engine-th SDMA engine the runtime reports for this direction (round-robin over them), forced onto SDMA
    uint32_t mask = 0;
    if (hsa_amd_memory_copy_engine_status(da, sa, &mask) != HSA_STATUS_SUCCESS || !mask) mask = 0x1u;
    int nset = 0;
    for (uint32_t b = 1; b; b <<= 1) nset += (mask & b) ? 1 : 0;
    int pick = engine % nset;
    uint32_t bit = 0;
    for (uint32_t b = 1; b; b <<= 1)
        if (mask & b) {
            if (pick == 0) { bit = b; break; }
            pick--;
        }
    hsa_status_t st = hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, bytes, 0, nullptr, sig,
                                                          (hsa_amd_sdma_engine_id_t)bit, true);
    if (st != HSA_STATUS_SUCCESS) {   // the reported engine refused: any SDMA engine
        for (uint32_t b = 1; b && b <= 0x8000u && st != HSA_STATUS_SUCCESS; b <<= 1)
            st = hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, bytes, 0, nullptr, sig,
                                                      (hsa_amd_sdma_engine_id_t)b, true);
    }
    if (st != HSA_STATUS_SUCCESS) {
        hsa_signal_destroy(sig);
        return fail(HUM_ERR_HIP, "hum_dma_copy: no SDMA engine accepted the copy");
    }
    ticket->signal = sig.handle;
    ticket->bytes = bytes;
    return HUM_OK;
}

extern "C" int hum_dma_wait(hum_dma_ticket* ticket) {
    if (!ticket || !ticket->signal) return fail(HUM_ERR_ARG, "hum_dma_wait: no copy in flight");
    hsa_signal_t sig;
    sig.handle = ticket->signal;
    // a chunk's pull takes 0.05-1 ms: spin for up to ~2 ms (no interrupt wake-up on the gather's critical path at
    // the end of a run), then sleep on the signal
    static const uint64_t spin = [] {
        uint64_t f = 0;
        return hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &f) == HSA_STATUS_SUCCESS && f ? f / 500 : 0;
    }();
    hsa_signal_value_t v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, spin, HSA_WAIT_STATE_ACTIVE);
    while (v >= 1)
        v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    hsa_signal_destroy(sig);
    ticket->signal = 0;
    if (v != 0) return fail(HUM_ERR_HIP, "hum_dma_wait: the copy engine reported an error");
    return HUM_OK;
}
