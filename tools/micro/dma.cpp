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
    if (hsa_amd_memory_copy_engine_status(da, sa, &mask) != HSA_STATUS_SUCCESS) return -4;
    hsa_signal_t sig;
    if (hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return -5;
    hsa_amd_sdma_engine_id_t eng = (hsa_amd_sdma_engine_id_t)engine_bit;
    if (!(mask & (uint32_t)engine_bit)) {   // the requested engine is busy / absent: take the lowest available one
        for (uint32_t b = 1; b; b <<= 1)
            if (mask & b) { eng = (hsa_amd_sdma_engine_id_t)b; break; }
    }
    hsa_status_t st = hsa_amd_memory_async_copy_on_engine(dst, da, src, sa, bytes, 0, nullptr, sig, eng, true);
    if (st != HSA_STATUS_SUCCESS) { hsa_signal_destroy(sig); return -6; }
    if (wait) hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
    hsa_signal_destroy(sig);
    return (int)mask;
}
