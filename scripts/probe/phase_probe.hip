// Phase-timestamp build of the ppo_loss forward (measurement only): s_memrealtime (100 MHz)
// per block at entry / after the token pass / after the block reduction / after arrival /
// after the partial fold / at the end, to see where the launch's time goes.
#define SKYRL_PHASE_PROBE
#include "../../skyrl_amd/csrc/capi.hip"
#include "../../skyrl_amd/csrc/ppo_loss.hip"

extern "C" int probe_read(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_phase), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int probe_clear() {
    static uint64_t zeros[8192 * 8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_phase), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
