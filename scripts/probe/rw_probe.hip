// Read+write ceiling probe (measurement only, not part of the product). Copies rows of V bf16
// (the fused training pass's traffic: V*2 read + V*2 written per token) with several
// structures, to find what limits policy_train_resident_kernel's 4.8 TB/s:
//   mode 0: grid-stride copy, U 16-B vectors in flight per thread (nt loads, nt|plain stores)
//   mode 1: one block per row, whole row loaded into registers, barrier, then stored
//           (policy_train_resident's shape: NT threads x NV vectors)
//   mode 2: mode 1 with the row split over 2 blocks (half rows, twice the blocks in flight)
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void st(u32x4* p, u32x4 v, int nts) {
    if (nts) __builtin_nontemporal_store(v, p);
    else *p = v;
}

template <int U>
__global__ __launch_bounds__(256) void copy_unroll(const u32x4* __restrict__ x, u32x4* __restrict__ y, int64_t n, int nts) {
    const int64_t step = (int64_t)gridDim.x * 256 * U;
    for (int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x; base < n; base += step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            v[u] = i < n ? __builtin_nontemporal_load(x + i) : u32x4{0, 0, 0, 0};
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + u * 256;
            if (i < n) st(y + i, v[u], nts);
        }
    }
}

template <int NT, int NV>
__global__ __launch_bounds__(NT) void copy_rows_resident(const u32x4* __restrict__ x, u32x4* __restrict__ y, int nvec_row,
                                                         int parts, int nts) {
    __shared__ uint32_t s_acc[NT / 64];
    const int row = blockIdx.x / parts, part = blockIdx.x % parts;
    const int per = (nvec_row + parts - 1) / parts;
    const int lo = part * per, hi = min(nvec_row, lo + per);
    const u32x4* r = x + (int64_t)row * nvec_row;
    u32x4* o = y + (int64_t)row * nvec_row;
    u32x4 v[NV];
    uint32_t acc = 0;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int i = lo + threadIdx.x + k * NT;
        v[k] = i < hi ? __builtin_nontemporal_load(r + i) : u32x4{0, 0, 0, 0};
        acc ^= v[k].x;
    }
    // a block-wide reduction + barrier between the sweeps, as the fused kernel has
    for (int off = 32; off > 0; off >>= 1) acc ^= __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0) s_acc[threadIdx.x / 64] = acc;
    __syncthreads();
    const uint32_t a0 = s_acc[0];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        const int i = lo + threadIdx.x + k * NT;
        asm volatile("" : "+v"(v[k]));
        if (i < hi) st(o + i, v[k] ^ u32x4{a0 & 0, 0, 0, 0}, nts);
    }
}

extern "C" int rw_probe(const void* x, void* y, int64_t rows, int V, int mode, int param, int nts, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    const int nvec_row = V / 8;
    const int64_t n = rows * nvec_row;
    if (mode == 0) {
        const int blocks = param;
        hipLaunchKernelGGL(copy_unroll<8>, dim3(blocks), dim3(256), 0, s, (const u32x4*)x, (u32x4*)y, n, nts);
    } else if (mode == 1) {
        if (param == 768)
            hipLaunchKernelGGL((copy_rows_resident<768, 25>), dim3(rows), dim3(768), 0, s, (const u32x4*)x, (u32x4*)y,
                               nvec_row, 1, nts);
        else
            hipLaunchKernelGGL((copy_rows_resident<1024, 19>), dim3(rows), dim3(1024), 0, s, (const u32x4*)x,
                               (u32x4*)y, nvec_row, 1, nts);
    } else if (mode == 2) {
        if (param == 384)
            hipLaunchKernelGGL((copy_rows_resident<384, 25>), dim3(rows * 2), dim3(384), 0, s, (const u32x4*)x,
                               (u32x4*)y, nvec_row, 2, nts);
        else
            hipLaunchKernelGGL((copy_rows_resident<256, 25>), dim3(rows * 3), dim3(256), 0, s, (const u32x4*)x,
                               (u32x4*)y, nvec_row, 3, nts);
    } else if (mode == 3) {
        hipLaunchKernelGGL(copy_unroll<4>, dim3(param), dim3(256), 0, s, (const u32x4*)x, (u32x4*)y, n, nts);
    } else if (mode == 4) {
        hipLaunchKernelGGL(copy_unroll<16>, dim3(param), dim3(256), 0, s, (const u32x4*)x, (u32x4*)y, n, nts);
    }
    return (int)hipGetLastError();
}
