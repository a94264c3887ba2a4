// a5: GAE advantage/return with masked whitening.
// Reference: compute_gae_advantage_return (skyrl-train/skyrl_train/utils/
// ppo_utils.py:1101-1129) + masked_whiten / masked_var (:148-172).
//
// Kernel 1: one wave per row. The reverse recurrence A_t = d_t + c*A_{t+1}
// (c = gamma*lambd, d_t = r_t + gamma*V_{t+1} - V_t, V_R := 0, no mask in the
// recursion) is an affine scan: each lane owns 4 consecutive steps of a
// 256-step tile, folds them to (mult, add), and the wave combines lanes with a
// log-step shuffle scan from the high lane down; tiles are walked from the end
// carrying A into the next tile; a lane issues the loads of 4 tiles (16-B vectors) before the
// first wait. returns = A + V. Each wave also emits the row's weighted Welford triple
// (sum m, mean, M2), from per-lane fp64 masked sums merged with Chan's formula.
// Kernel 2 (grid-wide, elementwise): every workgroup folds the N row triples
// (Chan's parallel formula, fp64, fixed order => identical in every block)
// into the masked mean and unbiased masked variance, then writes
// (A - mean) * rsqrt(var + 1e-8) for its slice; block 0 writes the status
// word (mask sum 0 or 1 => the reference's ValueError).
#include "common.h"

namespace skyrl {
namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerBlock = kThreads / kWave;
constexpr int kTile = kWave * 4;

struct RowStat {
    double w, mean, m2;
};

constexpr int kPreTiles = 4;  // tiles a lane loads before the first wait (R <= 1024: the whole row)

// Loads of one lane's 4 steps of a tile: r, V, mask and V at the step after the lane's last.
struct LaneTile {
    float r[4], v[4], m[4], vn;
};

__device__ __forceinline__ void load_tile(LaneTile& x, const float* __restrict__ rew, const float* __restrict__ val,
                                          const void* __restrict__ mask, int mask_dtype, int64_t base, int t0, int R,
                                          bool vec) {
    if (vec && t0 + 3 < R) {
        const float4 r4 = *reinterpret_cast<const float4*>(rew + base + t0);
        const float4 v4 = *reinterpret_cast<const float4*>(val + base + t0);
        x.r[0] = r4.x; x.r[1] = r4.y; x.r[2] = r4.z; x.r[3] = r4.w;
        x.v[0] = v4.x; x.v[1] = v4.y; x.v[2] = v4.z; x.v[3] = v4.w;
        load_mask4(mask, mask_dtype, base + t0, x.m);
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int t = t0 + k;
            x.r[k] = t < R ? rew[base + t] : 0.f;
            x.v[k] = t < R ? val[base + t] : 0.f;
            x.m[k] = t < R ? load_mask(mask, mask_dtype, base + t) : 0.f;
        }
    }
    x.vn = (t0 + 4 < R) ? val[base + t0 + 4] : 0.f;  // V_{t+1} of the lane's last step (V_R := 0)
}

__global__ __launch_bounds__(kThreads) void gae_scan_kernel(const float* __restrict__ rew, const float* __restrict__ val,
                                                            const void* __restrict__ mask, int mask_dtype, int N, int R,
                                                            float gamma, float lambd, bool vec, float* __restrict__ adv,
                                                            float* __restrict__ ret, RowStat* __restrict__ stats) {
    const int lane = threadIdx.x & (kWave - 1);
    const int row = blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
    if (row >= N) return;
    const int64_t base = (int64_t)row * R;
    const float c = gamma * lambd;
    float carry = 0.f;  // A_{tile_end}
    // masked sums of this lane (weights m): sum m, sum m*A, sum m*A^2 in fp64, turned into a
    // Welford triple at the end (the per-element Welford division was the scan's VALU pole)
    double sw = 0.0, s1 = 0.0, s2 = 0.0;
    const int ntiles = (R + kTile - 1) / kTile;
    for (int tb = ntiles - 1; tb >= 0; tb -= kPreTiles) {
        LaneTile x[kPreTiles];
#pragma unroll
        for (int u = 0; u < kPreTiles; ++u)
            if (tb - u >= 0) load_tile(x[u], rew, val, mask, mask_dtype, base, (tb - u) * kTile + lane * 4, R, vec);
#pragma unroll
        for (int u = 0; u < kPreTiles; ++u) {
            const int tile = tb - u;
            if (tile < 0) break;
            const int t0 = tile * kTile + lane * 4;
            float d[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float nv = k < 3 ? x[u].v[k + 1] : x[u].vn;
                d[k] = (t0 + k < R) ? (x[u].r[k] + gamma * nv) - x[u].v[k] : 0.f;
            }
            // lane-local fold from the end: A_t0 = add + mult * A_in
            float add = 0.f, mult = 1.f;
#pragma unroll
            for (int k = 3; k >= 0; --k) {
                if (t0 + k < R) {
                    add = d[k] + c * add;
                    mult = c * mult;
                }
            }
            // inclusive scan from high lanes to low lanes: compose (mult, add) maps.
            float sm = mult, sa = add;
#pragma unroll
            for (int off = 1; off < kWave; off <<= 1) {
                const float om = __shfl_down(sm, off, kWave);
                const float oa = __shfl_down(sa, off, kWave);
                if (lane + off < kWave) {
                    sa = sa + sm * oa;
                    sm = sm * om;
                }
            }
            // A entering this lane's block end = the next lane's inclusive value applied to carry
            float in_next = __shfl_down(sa + sm * carry, 1, kWave);
            if (lane == kWave - 1) in_next = carry;
            float a_cur = in_next;
            float A[4];
#pragma unroll
            for (int k = 3; k >= 0; --k) {
                if (t0 + k < R) {
                    a_cur = d[k] + c * a_cur;
                    A[k] = a_cur;
                } else {
                    A[k] = 0.f;
                }
            }
            carry = __shfl(sa + sm * carry, 0, kWave);
            if (vec && t0 + 3 < R) {
                *reinterpret_cast<float4*>(adv + base + t0) = make_float4(A[0], A[1], A[2], A[3]);
                *reinterpret_cast<float4*>(ret + base + t0) =
                    make_float4(A[0] + x[u].v[0], A[1] + x[u].v[1], A[2] + x[u].v[2], A[3] + x[u].v[3]);
            } else {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    if (t0 + k < R) {
                        adv[base + t0 + k] = A[k];
                        ret[base + t0 + k] = A[k] + x[u].v[k];
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const double m = (double)x[u].m[k], a = (double)A[k];
                sw += m;
                s1 = fma(m, a, s1);
                s2 = fma(m * a, a, s2);
            }
        }
    }
    // lane triple (w, mean, M2), then merge lanes (Chan)
    double w = sw, mean = 0.0, m2 = 0.0;
    if (sw > 0.0) {
        mean = s1 / sw;
        m2 = fmax(s2 - s1 * mean, 0.0);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const double ow = __shfl_xor(w, off, kWave);
        const double om = __shfl_xor(mean, off, kWave);
        const double om2 = __shfl_xor(m2, off, kWave);
        const double nw = w + ow;
        if (nw > 0.0) {
            const double delta = om - mean;
            mean = mean + delta * (ow / nw);
            m2 = m2 + om2 + delta * delta * (w * ow / nw);
        }
        w = nw;
    }
    if (lane == 0) stats[row] = RowStat{w, mean, m2};
}

__global__ __launch_bounds__(kThreads) void gae_whiten_kernel(float* __restrict__ adv, const RowStat* __restrict__ stats,
                                                              int N, int64_t total, bool vec,
                                                              int32_t* __restrict__ status) {
    __shared__ float s_mr[2];
    double w = 0.0, mean = 0.0, m2 = 0.0;
    if (threadIdx.x < kWave) {
        // lane-strided sequential fold, then a fixed shuffle tree: same order in every block
        for (int r = threadIdx.x; r < N; r += kWave) {
            const RowStat s = stats[r];
            const double nw = w + s.w;
            if (nw > 0.0) {
                const double delta = s.mean - mean;
                mean = mean + delta * (s.w / nw);
                m2 = m2 + s.m2 + delta * delta * (w * s.w / nw);
            }
            w = nw;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double ow = __shfl_xor(w, off, kWave);
            const double om = __shfl_xor(mean, off, kWave);
            const double om2 = __shfl_xor(m2, off, kWave);
            const double nw = w + ow;
            if (nw > 0.0) {
                const double delta = om - mean;
                mean = mean + delta * (ow / nw);
                m2 = m2 + om2 + delta * delta * (w * ow / nw);
            }
            w = nw;
        }
    }
    if (threadIdx.x == 0) {
        // masked_var: masked_mean(centered^2) * msum/(msum-1) = m2/(msum-1)
        const float mean_f = (float)mean;
        const float var_f = (w > 1.0) ? (float)(m2 / (w - 1.0)) : __builtin_nanf("");
        s_mr[0] = mean_f;
        s_mr[1] = 1.0f / sqrtf(var_f + 1e-8f);
        if (blockIdx.x == 0 && status) *status = (w == 0.0) ? 1 : ((w == 1.0) ? 2 : 0);
    }
    __syncthreads();
    const float mu = s_mr[0], rs = s_mr[1];
    if (vec) {  // total % 4 == 0, 16-B aligned: float4 grid-stride
        float4* a4 = reinterpret_cast<float4*>(adv);
        const int64_t n4 = total >> 2;
        for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
            float4 x = a4[i];
            a4[i] = make_float4((x.x - mu) * rs, (x.y - mu) * rs, (x.z - mu) * rs, (x.w - mu) * rs);
        }
        return;
    }
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads)
        adv[i] = (adv[i] - mu) * rs;
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" size_t skyrl_gae_workspace_bytes(int32_t N) { return (size_t)(N > 0 ? N : 1) * sizeof(RowStat) + 256; }

extern "C" int skyrl_gae_advantage_return(const float* rewards, const float* values, const void* response_mask,
                                          int mask_dtype, int32_t N, int32_t R, float gamma, float lambd,
                                          float* advantages, float* returns, void* workspace, int32_t* status,
                                          void* stream) {
    SKYRL_REQUIRE(N > 0 && R > 0, "gae: empty batch");
    SKYRL_REQUIRE(rewards && values && response_mask && advantages && returns && workspace, "gae: null pointer");
    RowStat* stats = reinterpret_cast<RowStat*>(workspace);
    hipStream_t s = as_stream(stream);
    const auto a16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
    const bool vec = (R % 4) == 0 && a16(rewards) && a16(values) && a16(advantages) && a16(returns) &&
                     (mask_dtype == SKYRL_U8 ? (reinterpret_cast<uintptr_t>(response_mask) & 3) == 0
                                             : a16(response_mask));
    hipLaunchKernelGGL(gae_scan_kernel, dim3((N + kRowsPerBlock - 1) / kRowsPerBlock), dim3(kThreads), 0, s, rewards,
                       values, response_mask, mask_dtype, N, R, gamma, lambd, vec, advantages, returns, stats);
    int rc = check_launch("gae_scan_kernel");
    if (rc) return rc;
    const int64_t total = (int64_t)N * R;
    int64_t blocks = (total + kThreads * 8 - 1) / (kThreads * 8);
    if (blocks > 1024) blocks = 1024;
    if (blocks < 1) blocks = 1;
    const bool vec_w = (total % 4) == 0 && a16(advantages);
    hipLaunchKernelGGL(gae_whiten_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, s, advantages, stats, N, total,
                       vec_w, status);
    return check_launch("gae_whiten_kernel");
}
