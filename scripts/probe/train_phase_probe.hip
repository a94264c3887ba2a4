// Phase-timestamp build of the fused training pass (measurement only): s_memrealtime (100 MHz)
// per block at entry / end of sweep 1 / after the first barrier / after the second barrier /
// end of sweep 2, plus the CU id, to see where a row's time goes.
#define SKYRL_TRAIN_PHASE_PROBE
#include "../../skyrl_amd/csrc/capi.hip"
#include "../../skyrl_amd/csrc/policy_train.hip"

extern "C" int probe_read(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_tphase), bytes, 0, hipMemcpyDeviceToHost);
}
