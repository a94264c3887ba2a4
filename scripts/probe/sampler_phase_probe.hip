// Phase-timestamp build of the sampler (measurement only): s_memrealtime (100 MHz) per row
// workgroup at entry / after the first iteration (and the seeding barrier) / end of wave 0's
// stream / after the workgroup's final barrier / before the token write, plus the CU id.
#define SKYRL_SAMPLER_PHASE_PROBE
#include "../../skyrl_amd/csrc/capi.hip"
#include "../../skyrl_amd/csrc/sampler.hip"

extern "C" int probe_read(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_sphase), bytes, 0, hipMemcpyDeviceToHost);
}

extern "C" void probe_set_row(int v) { skyrl::g_sampler_row = v; }

extern "C" int probe_clear() {
    static uint64_t zeros[4096 * 8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sphase), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
