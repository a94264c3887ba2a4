// Phase-timestamp build of the lm_head GEMM (measurement only): s_memrealtime (100 MHz) per tile
// workgroup at entry / end of the K loop / image written / end of sampler pass 1 / end of the
// candidate evaluation / before the partial write.
#define SKYRL_GEMM_PHASE_PROBE
#include "../../skyrl_amd/csrc/capi.hip"
#include "../../skyrl_amd/csrc/lmhead_gemm.hip"

extern "C" int probe_read(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gphase), bytes, 0, hipMemcpyDeviceToHost);
}
// the probe library has no skyrl_lmhead_state_merge (logprob epilogue unused here)
extern "C" int skyrl_lmhead_state_merge(const void*, int32_t, int32_t, float*, float*, float*, void*) { return 1; }
