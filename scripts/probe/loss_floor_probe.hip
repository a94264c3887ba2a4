// Floor probe for the advantage+loss leg (measurement only, not part of the product): what a
// graph node of the fused loss's shape costs with less and less work. 512 blocks x 256 threads,
// 4 tokens per thread (one 1024-column row chunk per block):
//   mode 0: empty kernel
//   mode 1: 4 float4 loads per thread (lp, old, mask, ref), one float4 store
//   mode 2: mode 1 + block reduction of 5 partials + a 5-float record store
//   mode 3: one block folding 512 x 5 records (the finish's fold), no other blocks
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ __launch_bounds__(256) void floor_kernel(const float4* __restrict__ a, const float4* __restrict__ b,
                                                    const float4* __restrict__ c, const float4* __restrict__ d,
                                                    float4* __restrict__ out, float* __restrict__ rec, int mode) {
    __shared__ float s[4 * 5];
    if (mode == 0) return;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (mode == 3) {
        if (blockIdx.x) return;
        double t[5] = {0, 0, 0, 0, 0};
        for (int k = 0; k < 5; ++k) t[k] = (double)rec[k * 512 + threadIdx.x] + (double)rec[k * 512 + 256 + threadIdx.x];
        for (int k = 0; k < 5; ++k)
            for (int off = 32; off > 0; off >>= 1) t[k] += __shfl_xor(t[k], off, 64);
        if ((threadIdx.x & 63) == 0)
            for (int k = 0; k < 5; ++k) s[(threadIdx.x >> 6) * 5 + k] = (float)t[k];
        __syncthreads();
        if (threadIdx.x < 5) rec[4096 + threadIdx.x] = s[threadIdx.x] + s[5 + threadIdx.x] + s[10 + threadIdx.x] + s[15 + threadIdx.x];
        return;
    }
    const float4 x = a[i], y = b[i], z = c[i], w = d[i];
    float4 o;
    o.x = x.x * y.x + z.x * w.x;
    o.y = x.y * y.y + z.y * w.y;
    o.z = x.z * y.z + z.z * w.z;
    o.w = x.w * y.w + z.w * w.w;
    out[i] = o;
    if (mode == 1) return;
    float v[5] = {o.x, o.y, o.z, o.w, x.x};
    for (int k = 0; k < 5; ++k)
        for (int off = 32; off > 0; off >>= 1) v[k] += __shfl_xor(v[k], off, 64);
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < 5; ++k) s[(threadIdx.x >> 6) * 5 + k] = v[k];
    __syncthreads();
    if (threadIdx.x < 5) rec[threadIdx.x * 512 + blockIdx.x] = s[threadIdx.x] + s[5 + threadIdx.x] + s[10 + threadIdx.x] + s[15 + threadIdx.x];
}

extern "C" int floor_probe(const void* a, const void* b, const void* c, const void* d, void* out, void* rec, int mode,
                           void* stream) {
    hipLaunchKernelGGL(floor_kernel, dim3(512), dim3(256), 0, (hipStream_t)stream, (const float4*)a, (const float4*)b,
                       (const float4*)c, (const float4*)d, (float4*)out, (float*)rec, mode);
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
