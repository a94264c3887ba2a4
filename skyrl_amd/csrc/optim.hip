// a12/a14: learner optimizer step over a flat fp32 parameter shard.
//
// Reference semantics (skyrl-train/skyrl_train/):
//   PolicyWorkerBase.optim_step        workers/worker.py:900-925 (grads *= 1/n_micro)
//   FSDPStrategy.optimizer_step        distributed/fsdp_strategy.py:160-190 (clip_grad_norm_
//                                      with max_norm; non-finite norm => zero_grad, no step)
//   fsdp2_clip_grad_norm_              distributed/fsdp_utils.py:388-401 (torch
//                                      _get_total_norm + _clip_grads_with_norm_:
//                                      coef = clamp(max_norm / (norm + 1e-6), max=1))
//   optim.AdamW(lr, betas, wd)         distributed/fsdp_strategy.py:284-296 (torch foreach
//                                      AdamW: p *= 1-lr*wd; m.lerp_(g, 1-b1);
//                                      v = v*b2 + (1-b2)*g*g; p += -lr/bc1 * m/(sqrt(v)/sqrt(bc2)+eps))
//
// Three launches, no host synchronisation:
//   sumsq_partial_kernel / sumsq_fold_kernel  sum of squares of the shard (fixed grid and
//       fixed fold order => deterministic). Under DP sharding the host all-reduces this one
//       scalar over RCCL before the plan.
//   adamw_plan_kernel (1 thread)  grad norm, clip coefficient, finiteness, step counter and
//       bias corrections -> a 6-float plan in device memory.
//   adamw_update_kernel  one HBM pass over (p, g, m, v): 16 B read + 12 B written per
//       parameter, + 2 B when the bf16 copy for the rollout engine is written in the same
//       pass (the colocated learner->rollout weight sync of a14 costs no extra read).
#include "common.h"

namespace skyrl {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kMaxPartials = 2048;

// PLAN_UNIFORM (per-parameter form only): every parameter is updated this step and all share one
// step count, so the update pass runs the plain loop on PLAN_STEP / PLAN_BC2SQRT
enum { PLAN_SKIP = 0, PLAN_GMUL, PLAN_DECAY, PLAN_STEP, PLAN_BC2SQRT, PLAN_EPS, PLAN_UNIFORM, PLAN_N };
constexpr int kSegTile = kThreads * 4;  // elements per tile of the per-parameter segment map

__host__ __device__ inline int sumsq_blocks(int64_t n) {
    const int64_t per_block = (int64_t)kThreads * 4 * 8;  // 8 float4 per thread at least
    int64_t b = (n + per_block - 1) / per_block;
    if (b < 1) b = 1;
    if (b > kMaxPartials) b = kMaxPartials;
    return (int)b;
}

__global__ __launch_bounds__(kThreads) void sumsq_partial_kernel(const float* __restrict__ x, int64_t n,
                                                                  double* __restrict__ partials) {
    __shared__ double lds[kThreads / kWave];
    const int64_t n4 = n >> 2;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    float a0 = 0.f, a1 = 0.f;
    int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    for (; i + stride < n4; i += 2 * stride) {
        const f32x4 u = __builtin_nontemporal_load(x4 + i);
        const f32x4 w = __builtin_nontemporal_load(x4 + i + stride);
        a0 += u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w;
        a1 += w.x * w.x + w.y * w.y + w.z * w.z + w.w * w.w;
    }
    if (i < n4) {
        const f32x4 u = __builtin_nontemporal_load(x4 + i);
        a0 += u.x * u.x + u.y * u.y + u.z * u.z + u.w * u.w;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const float t = x[(n4 << 2) + threadIdx.x];
        a1 += t * t;
    }
    double s = wave_sum((double)a0 + (double)a1);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    if (lane == 0) lds[w] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < kThreads / kWave; ++k) t += lds[k];
        partials[blockIdx.x] = t;
    }
}

__global__ __launch_bounds__(kThreads) void sumsq_fold_kernel(const double* __restrict__ partials, int nb,
                                                               float* __restrict__ out) {
    __shared__ double lds[kThreads / kWave];
    double s = 0.0;
    for (int k = threadIdx.x; k < nb; k += kThreads) s += partials[k];
    s = wave_sum(s);
    const int lane = threadIdx.x & (kWave - 1), w = threadIdx.x / kWave;
    if (lane == 0) lds[w] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < kThreads / kWave; ++k) t += lds[k];
        out[0] = (float)t;
    }
}

__global__ void adamw_plan_kernel(const float* __restrict__ sumsq, skyrl_adamw_params hp, int32_t* step_count,
                                  float* __restrict__ plan, float* __restrict__ grad_norm_out) {
    // norm of the 1/n_micro-scaled gradient (the reference scales before clipping)
    const float norm = sqrtf(fmaxf(sumsq[0], 0.f)) * hp.grad_scale;
    if (grad_norm_out) grad_norm_out[0] = norm;
    float coef = 1.f;
    if (hp.max_grad_norm > 0.f) coef = fminf(hp.max_grad_norm / (norm + 1e-6f), 1.f);
    const bool finite = isfinite(norm) || hp.max_grad_norm <= 0.f;
    if (!finite) {  // fsdp_strategy.py:178-186: zero_grad and return, step not taken
        plan[PLAN_SKIP] = 1.f;
        return;
    }
    const int step = step_count[0] + 1;
    step_count[0] = step;
    const double bc1 = 1.0 - pow((double)hp.beta1, (double)step);
    const double bc2 = 1.0 - pow((double)hp.beta2, (double)step);
    plan[PLAN_SKIP] = 0.f;
    plan[PLAN_GMUL] = hp.grad_scale * coef;
    plan[PLAN_DECAY] = 1.f - hp.lr * hp.weight_decay;
    plan[PLAN_STEP] = (float)(-((double)hp.lr / bc1));
    plan[PLAN_BC2SQRT] = (float)sqrt(bc2);
    plan[PLAN_EPS] = hp.eps;
    plan[PLAN_UNIFORM] = 1.f;
}

// Per-parameter plan (torch.optim.AdamW over a module: a parameter whose .grad is None is
// skipped and its own `step` state is not advanced, so its bias corrections follow its own count).
// One workgroup: the global clip / finiteness as adamw_plan_kernel, then per parameter p
// (touched[p] = some rank's backward reached it since the last step): step[p] += 1 and
// coef[2p..2p+1] = (-lr / bc1(step[p]), sqrt(bc2(step[p]))), or (0, 0) = leave p untouched.
// PLAN_UNIFORM = every parameter touched and all counts equal (the update then runs the plain
// loop on coef[0..1] as PLAN_STEP / PLAN_BC2SQRT). Otherwise (a parameter skipped once, or never
// touched) the update reads one coefficient pair per 16-B vector and skips untouched vectors
// without loading them; only vectors that straddle a parameter boundary go element by element.
__global__ __launch_bounds__(kThreads) void adamw_seg_plan_kernel(const float* __restrict__ sumsq,
                                                                   skyrl_adamw_params hp,
                                                                   const int32_t* __restrict__ touched, int nparams,
                                                                   int32_t* __restrict__ pstep, float* __restrict__ plan,
                                                                   float* __restrict__ coef,
                                                                   float* __restrict__ grad_norm_out) {
    const float norm = sqrtf(fmaxf(sumsq[0], 0.f)) * hp.grad_scale;
    float clip = 1.f;
    if (hp.max_grad_norm > 0.f) clip = fminf(hp.max_grad_norm / (norm + 1e-6f), 1.f);
    const bool finite = isfinite(norm) || hp.max_grad_norm <= 0.f;
    if (threadIdx.x == 0 && grad_norm_out) grad_norm_out[0] = norm;
    if (!finite) {  // fsdp_strategy.py:178-186: no step, no count advanced
        if (threadIdx.x == 0) plan[PLAN_SKIP] = 1.f;
        return;
    }
    __shared__ int s_first;
    if (threadIdx.x == 0) s_first = touched[0] ? pstep[0] + 1 : -1;
    __syncthreads();
    const int first = s_first;
    int uniform = 1;
    for (int p = threadIdx.x; p < nparams; p += kThreads) {
        if (touched[p]) {
            const int step = pstep[p] + 1;
            pstep[p] = step;
            const double bc1 = 1.0 - pow((double)hp.beta1, (double)step);
            const double bc2 = 1.0 - pow((double)hp.beta2, (double)step);
            coef[2 * p] = (float)(-((double)hp.lr / bc1));
            coef[2 * p + 1] = (float)sqrt(bc2);
            uniform &= step == first;
        } else {
            coef[2 * p] = 0.f;
            coef[2 * p + 1] = 0.f;
            uniform = 0;
        }
    }
    uniform = __syncthreads_and(uniform);
    if (threadIdx.x == 0) {
        plan[PLAN_SKIP] = 0.f;
        plan[PLAN_GMUL] = hp.grad_scale * clip;
        plan[PLAN_DECAY] = 1.f - hp.lr * hp.weight_decay;
        plan[PLAN_EPS] = hp.eps;
        plan[PLAN_UNIFORM] = uniform ? 1.f : 0.f;
        if (uniform) {  // the plain loop's constants: every parameter's (equal) step
            const double bc1 = 1.0 - pow((double)hp.beta1, (double)first);
            const double bc2 = 1.0 - pow((double)hp.beta2, (double)first);
            plan[PLAN_STEP] = (float)(-((double)hp.lr / bc1));
            plan[PLAN_BC2SQRT] = (float)sqrt(bc2);
        }
    }
}

struct AdamPlan {
    float gmul, decay, step, bc2s, eps, omb1, b2, omb2;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamPlan& a) {
    g *= a.gmul;
    p *= a.decay;
    m = m + a.omb1 * (g - m);               // lerp(m, g, 1-b1), weight < 0.5 branch
    v = v * a.b2 + a.omb2 * g * g;          // mul_(b2).addcmul_(g, g, 1-b2)
    const float denom = sqrtf(v) / a.bc2s + a.eps;
    p = p + a.step * (m / denom);           // addcdiv_(m, denom, value=-lr/bc1)
}

// The per-parameter segment map of a shard: segment s covers shard elements [start[s], start[s+1])
// of parameter owner[s] (segments cover the shard, padding included); tile_seg[t] = the segment
// holding element t * kSegTile. Elements of an untouched parameter (coef (0, 0)) are left as they
// are; a vector none of whose elements is updated is not stored.
struct SegMap {
    const int64_t* start;
    const int32_t* owner;
    const int32_t* tile_seg;
    const float* coef;
};

__device__ __forceinline__ int seg_of(const SegMap& sm, int s, int64_t e) {
    while (sm.start[s + 1] <= e) ++s;
    return s;
}

template <bool SHADOW>
__device__ void adamw_seg_loop(float* __restrict__ param, const float* __restrict__ grad, float* __restrict__ exp_avg,
                               float* __restrict__ exp_avg_sq, uint16_t* __restrict__ shadow, int64_t n, AdamPlan a,
                               const SegMap& sm) {
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    f32x4* p4 = reinterpret_cast<f32x4*>(param);
    const f32x4* g4 = reinterpret_cast<const f32x4*>(grad);
    f32x4* m4 = reinterpret_cast<f32x4*>(exp_avg);
    f32x4* v4 = reinterpret_cast<f32x4*>(exp_avg_sq);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += stride) {
        int s = seg_of(sm, sm.tile_seg[(i << 2) / kSegTile], i << 2);
        if (sm.start[s + 1] >= (i << 2) + 4) {
            // the whole vector in one segment (all but the vectors that straddle a parameter
            // boundary): one coefficient lookup; an untouched parameter's vector is neither loaded
            // nor stored, so a step that skipped some parameters costs what the plain loop does
            const int o = sm.owner[s];
            const float st = sm.coef[2 * o], b2s = sm.coef[2 * o + 1];
            if (b2s == 0.f) continue;
            AdamPlan b = a;
            b.step = st;
            b.bc2s = b2s;
            const f32x4 pv = p4[i];
            const f32x4 gv = __builtin_nontemporal_load(g4 + i);
            const f32x4 mv = m4[i];
            const f32x4 vv = v4[i];
            float p[4] = {pv.x, pv.y, pv.z, pv.w}, m[4] = {mv.x, mv.y, mv.z, mv.w}, v[4] = {vv.x, vv.y, vv.z, vv.w};
            const float g[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) adam_elem(p[k], g[k], m[k], v[k], b);
            p4[i] = f32x4{p[0], p[1], p[2], p[3]};
            __builtin_nontemporal_store(f32x4{m[0], m[1], m[2], m[3]}, m4 + i);
            __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, v4 + i);
            if (SHADOW) {
                uint2 sh;
                sh.x = pack_bf16x2(p[0], p[1]);
                sh.y = pack_bf16x2(p[2], p[3]);
                reinterpret_cast<uint2*>(shadow)[i] = sh;
            }
            continue;
        }
        const f32x4 pv = p4[i];
        const f32x4 gv = __builtin_nontemporal_load(g4 + i);
        const f32x4 mv = m4[i];
        const f32x4 vv = v4[i];
        float p[4] = {pv.x, pv.y, pv.z, pv.w}, m[4] = {mv.x, mv.y, mv.z, mv.w}, v[4] = {vv.x, vv.y, vv.z, vv.w};
        const float g[4] = {gv.x, gv.y, gv.z, gv.w};
        bool any = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            s = seg_of(sm, s, (i << 2) + k);
            const int o = sm.owner[s];
            const float st = sm.coef[2 * o], b2s = sm.coef[2 * o + 1];
            if (b2s != 0.f) {
                AdamPlan b = a;
                b.step = st;
                b.bc2s = b2s;
                adam_elem(p[k], g[k], m[k], v[k], b);
                any = true;
            }
        }
        if (!any) continue;
        p4[i] = f32x4{p[0], p[1], p[2], p[3]};
        __builtin_nontemporal_store(f32x4{m[0], m[1], m[2], m[3]}, m4 + i);
        __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, v4 + i);
        if (SHADOW) {
            uint2 sh;
            sh.x = pack_bf16x2(p[0], p[1]);
            sh.y = pack_bf16x2(p[2], p[3]);
            reinterpret_cast<uint2*>(shadow)[i] = sh;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const int64_t k = (n4 << 2) + threadIdx.x;
        const int s = seg_of(sm, sm.tile_seg[k / kSegTile], k);
        const int o = sm.owner[s];
        if (sm.coef[2 * o + 1] == 0.f) return;
        AdamPlan b = a;
        b.step = sm.coef[2 * o];
        b.bc2s = sm.coef[2 * o + 1];
        float pk = param[k], mk = exp_avg[k], vk = exp_avg_sq[k];
        adam_elem(pk, grad[k], mk, vk, b);
        param[k] = pk;
        exp_avg[k] = mk;
        exp_avg_sq[k] = vk;
        if (SHADOW) shadow[k] = f32_to_bf16(pk);
    }
}

template <bool SHADOW>
__global__ __launch_bounds__(kThreads) void adamw_update_kernel(float* __restrict__ param, const float* __restrict__ grad,
                                                                 float* __restrict__ exp_avg, float* __restrict__ exp_avg_sq,
                                                                 uint16_t* __restrict__ shadow, int64_t n,
                                                                 const float* __restrict__ plan, float beta1, float beta2,
                                                                 SegMap sm) {
    if (plan[PLAN_SKIP] != 0.f) return;
    AdamPlan a;
    a.gmul = plan[PLAN_GMUL];
    a.decay = plan[PLAN_DECAY];
    a.step = plan[PLAN_STEP];
    a.bc2s = plan[PLAN_BC2SQRT];
    a.eps = plan[PLAN_EPS];
    a.omb1 = 1.f - beta1;
    a.b2 = beta2;
    a.omb2 = 1.f - beta2;
    if (sm.start && plan[PLAN_UNIFORM] == 0.f) {  // some parameter skipped or behind: per-parameter loop
        adamw_seg_loop<SHADOW>(param, grad, exp_avg, exp_avg_sq, shadow, n, a, sm);
        return;
    }
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    f32x4* p4 = reinterpret_cast<f32x4*>(param);
    const f32x4* g4 = reinterpret_cast<const f32x4*>(grad);
    f32x4* m4 = reinterpret_cast<f32x4*>(exp_avg);
    f32x4* v4 = reinterpret_cast<f32x4*>(exp_avg_sq);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += stride) {
        const f32x4 pv = p4[i];
        const f32x4 gv = __builtin_nontemporal_load(g4 + i);
        const f32x4 mv = m4[i];
        const f32x4 vv = v4[i];
        float p[4] = {pv.x, pv.y, pv.z, pv.w}, m[4] = {mv.x, mv.y, mv.z, mv.w}, v[4] = {vv.x, vv.y, vv.z, vv.w};
        const float g[4] = {gv.x, gv.y, gv.z, gv.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) adam_elem(p[k], g[k], m[k], v[k], a);
        p4[i] = f32x4{p[0], p[1], p[2], p[3]};
        __builtin_nontemporal_store(f32x4{m[0], m[1], m[2], m[3]}, m4 + i);
        __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, v4 + i);
        if (SHADOW) {
            uint2 s;
            s.x = pack_bf16x2(p[0], p[1]);
            s.y = pack_bf16x2(p[2], p[3]);
            reinterpret_cast<uint2*>(shadow)[i] = s;
        }
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const int64_t k = (n4 << 2) + threadIdx.x;
        float p = param[k], m = exp_avg[k], v = exp_avg_sq[k];
        adam_elem(p, grad[k], m, v, a);
        param[k] = p;
        exp_avg[k] = m;
        exp_avg_sq[k] = v;
        if (SHADOW) shadow[k] = f32_to_bf16(p);
    }
}

__global__ __launch_bounds__(kThreads) void cast_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y,
                                                              int64_t n) {
    const int64_t n4 = n >> 2;
    const int64_t stride = (int64_t)gridDim.x * kThreads;
    const f32x4* x4 = reinterpret_cast<const f32x4*>(x);
    for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < n4; i += stride) {
        const f32x4 p = __builtin_nontemporal_load(x4 + i);
        uint2 s;
        s.x = pack_bf16x2(p.x, p.y);
        s.y = pack_bf16x2(p.z, p.w);
        reinterpret_cast<uint2*>(y)[i] = s;
    }
    if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
        const int64_t k = (n4 << 2) + threadIdx.x;
        y[k] = f32_to_bf16(x[k]);
    }
}

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline unsigned stream_blocks(int64_t n) {
    int64_t b = ((n >> 2) + kThreads - 1) / kThreads;
    if (b > 8192) b = 8192;  // 32 waves per CU over 256 CUs; grid-stride beyond
    if (b < 1) b = 1;
    return (unsigned)b;
}

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" size_t skyrl_sumsq_workspace_bytes(int64_t n) { return sizeof(double) * (size_t)sumsq_blocks(n); }

extern "C" int skyrl_sumsq(const float* x, int64_t n, float* sumsq_out, void* workspace, void* stream) {
    SKYRL_REQUIRE(n >= 0, "sumsq: n < 0");
    SKYRL_REQUIRE(sumsq_out && workspace, "sumsq: null output/workspace");
    SKYRL_REQUIRE(n == 0 || (x && aligned16(x)), "sumsq: x null or not 16-byte aligned");
    const int nb = sumsq_blocks(n);
    hipStream_t s = as_stream(stream);
    double* partials = reinterpret_cast<double*>(workspace);
    if (n > 0) {
        hipLaunchKernelGGL(sumsq_partial_kernel, dim3(nb), dim3(kThreads), 0, s, x, n, partials);
    } else {
        (void)hipMemsetAsync(partials, 0, sizeof(double), s);
    }
    hipLaunchKernelGGL(sumsq_fold_kernel, dim3(1), dim3(kThreads), 0, s, partials, n > 0 ? nb : 1, sumsq_out);
    return check_launch("sumsq_kernel");
}

extern "C" int skyrl_adamw_plan(const float* sumsq, const skyrl_adamw_params* hp, int32_t* step_count, float* plan,
                                float* grad_norm_out, void* stream) {
    SKYRL_REQUIRE(sumsq && hp && step_count && plan, "adamw_plan: null pointer");
    SKYRL_REQUIRE(hp->lr >= 0.f && hp->eps >= 0.f && hp->beta1 >= 0.f && hp->beta1 < 1.f && hp->beta2 >= 0.f &&
                      hp->beta2 < 1.f,
                  "adamw_plan: invalid hyper-parameters");
    hipLaunchKernelGGL(adamw_plan_kernel, dim3(1), dim3(1), 0, as_stream(stream), sumsq, *hp, step_count, plan,
                       grad_norm_out);
    return check_launch("adamw_plan_kernel");
}

extern "C" size_t skyrl_adamw_plan_floats(void) { return PLAN_N; }

extern "C" int skyrl_adamw_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, void* param_bf16,
                                  int64_t n, const float* plan, float beta1, float beta2, void* stream) {
    SKYRL_REQUIRE(n >= 0, "adamw_update: n < 0");
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(param && grad && exp_avg && exp_avg_sq && plan, "adamw_update: null pointer");
    SKYRL_REQUIRE(aligned16(param) && aligned16(grad) && aligned16(exp_avg) && aligned16(exp_avg_sq),
                  "adamw_update: fp32 buffers must be 16-byte aligned");
    SKYRL_REQUIRE(!param_bf16 || (reinterpret_cast<uintptr_t>(param_bf16) & 7) == 0,
                  "adamw_update: bf16 copy must be 8-byte aligned");
    const unsigned nb = stream_blocks(n);
    hipStream_t s = as_stream(stream);
    const SegMap none{nullptr, nullptr, nullptr, nullptr};
    if (param_bf16) {
        hipLaunchKernelGGL(adamw_update_kernel<true>, dim3(nb), dim3(kThreads), 0, s, param, grad, exp_avg, exp_avg_sq,
                           reinterpret_cast<uint16_t*>(param_bf16), n, plan, beta1, beta2, none);
    } else {
        hipLaunchKernelGGL(adamw_update_kernel<false>, dim3(nb), dim3(kThreads), 0, s, param, grad, exp_avg,
                           exp_avg_sq, nullptr, n, plan, beta1, beta2, none);
    }
    return check_launch("adamw_update_kernel");
}

extern "C" size_t skyrl_adamw_seg_tile(void) { return kSegTile; }

extern "C" int skyrl_adamw_seg_plan(const float* sumsq, const skyrl_adamw_params* hp, const int32_t* touched,
                                    int32_t nparams, int32_t* param_step, float* plan, float* coef,
                                    float* grad_norm_out, void* stream) {
    SKYRL_REQUIRE(sumsq && hp && touched && param_step && plan && coef, "adamw_seg_plan: null pointer");
    SKYRL_REQUIRE(nparams >= 1, "adamw_seg_plan: nparams < 1");
    SKYRL_REQUIRE(hp->lr >= 0.f && hp->eps >= 0.f && hp->beta1 >= 0.f && hp->beta1 < 1.f && hp->beta2 >= 0.f &&
                      hp->beta2 < 1.f,
                  "adamw_seg_plan: invalid hyper-parameters");
    hipLaunchKernelGGL(adamw_seg_plan_kernel, dim3(1), dim3(kThreads), 0, as_stream(stream), sumsq, *hp, touched,
                       nparams, param_step, plan, coef, grad_norm_out);
    return check_launch("adamw_seg_plan_kernel");
}

extern "C" int skyrl_adamw_seg_update(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                      void* param_bf16, int64_t n, const float* plan, const float* coef,
                                      const int64_t* seg_start, const int32_t* seg_owner, int32_t nseg,
                                      const int32_t* tile_seg, float beta1, float beta2, void* stream) {
    SKYRL_REQUIRE(n >= 0, "adamw_seg_update: n < 0");
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(param && grad && exp_avg && exp_avg_sq && plan && coef && seg_start && seg_owner && tile_seg,
                  "adamw_seg_update: null pointer");
    SKYRL_REQUIRE(nseg >= 1, "adamw_seg_update: nseg < 1");
    SKYRL_REQUIRE(aligned16(param) && aligned16(grad) && aligned16(exp_avg) && aligned16(exp_avg_sq),
                  "adamw_seg_update: fp32 buffers must be 16-byte aligned");
    SKYRL_REQUIRE(!param_bf16 || (reinterpret_cast<uintptr_t>(param_bf16) & 7) == 0,
                  "adamw_seg_update: bf16 copy must be 8-byte aligned");
    const unsigned nb = stream_blocks(n);
    hipStream_t s = as_stream(stream);
    const SegMap sm{seg_start, seg_owner, tile_seg, coef};
    if (param_bf16) {
        hipLaunchKernelGGL(adamw_update_kernel<true>, dim3(nb), dim3(kThreads), 0, s, param, grad, exp_avg, exp_avg_sq,
                           reinterpret_cast<uint16_t*>(param_bf16), n, plan, beta1, beta2, sm);
    } else {
        hipLaunchKernelGGL(adamw_update_kernel<false>, dim3(nb), dim3(kThreads), 0, s, param, grad, exp_avg,
                           exp_avg_sq, nullptr, n, plan, beta1, beta2, sm);
    }
    return check_launch("adamw_update_kernel");
}

extern "C" int skyrl_cast_bf16(const float* x, void* y, int64_t n, void* stream) {
    SKYRL_REQUIRE(n >= 0, "cast_bf16: n < 0");
    if (n == 0) return SKYRL_OK;
    SKYRL_REQUIRE(x && y && aligned16(x) && (reinterpret_cast<uintptr_t>(y) & 7) == 0,
                  "cast_bf16: null or misaligned pointer");
    hipLaunchKernelGGL(cast_bf16_kernel, dim3(stream_blocks(n)), dim3(kThreads), 0, as_stream(stream), x,
                       reinterpret_cast<uint16_t*>(y), n);
    return check_launch("cast_bf16_kernel");
}
