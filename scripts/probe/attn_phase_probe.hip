// Per-wave timestamp build of the paged decode kernel (measurement only): s_memrealtime
// (100 MHz) at entry / after the first block's QK MFMA / after the block loop, plus the
// partition's token count and the CU / XCC id.
#define SKYRL_ATTN_PHASE_PROBE
#include "../../skyrl_amd/csrc/capi.hip"
#include "../../skyrl_amd/csrc/attention.hip"

extern "C" int probe_read(void* host, size_t bytes) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_aphase), bytes, 0, hipMemcpyDeviceToHost);
}
extern "C" int probe_clear() {
    static uint64_t zeros[8192 * 8];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_aphase), zeros, sizeof(zeros), 0, hipMemcpyHostToDevice);
}
