// Diagnostic helper (tools/micro/overlap.py): one device-to-device copy forced onto an SDMA engine through the HSA
// runtime (hsa_amd_memory_async_copy_on_engine), the engine the copy queue of a DMA transport would use, so the
// probe can tell whether a copy engine transfer overlaps the env kernel (which holds every CU's registers and LDS).
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

extern "C" int dma_copy(void* dst, const void* src, unsigned long long bytes, int engine_bit, int wait) {
    static bool inited = false;
    if (!inited) {
        if (hsa_init() != HSA_STATUS_SUCCESS) return -1;
        inited = true;
    }
    hsa_amd_pointer_info_t pi{};
    pi.size = sizeof(pi);
    if (hsa_amd_pointer_info(const_cast<void*>(src), &pi, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return -2;
    hsa_agent_t sa = pi.agentOwner;
    hsa_amd_pointer_info_t pd{};
    pd.size = sizeof(pd);
    if (hsa_amd_pointer_info(dst, &pd, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS) return -3;
    hsa_agent_t da = pd.agentOwner;
    uint32_t mask = 0;
    const hsa_status_t ms = hsa_amd_memory_copy_engine_status(da, sa, &mask);   // may refuse a same-agent pair
    hsa_signal_t sig;
    if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return -5;
    hsa_status_t st = HSA_STATUS_ERROR;
    for (uint32_t b = (uint32_t)engine_bit; b && b <= 0x8000u; b <<= 1) {   // the requested engine, else the next ones
        if (ms == HSA_STATUS_SUCCESS && mask && !(mask & b)) continue;
        st = hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, bytes, 0, nullptr, sig, (hsa_amd_sdma_engine_id_t)b,
                                                 true);
        if (st == HSA_STATUS_SUCCESS) break;
    }
    if (st != HSA_STATUS_SUCCESS) { hsa_signal_destroy(sig); return -6; }
    if (wait) hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    hsa_signal_destroy(sig);
    return ms == HSA_STATUS_SUCCESS ? (int)mask : 0;
}
