// lm_head-fused logprob + entropy. The [T,V] logits are never materialized.
//
// Reference: HFModelWrapper.forward, model_wrapper.py:308-363. The model's lm_head GEMM writes
// logits [n,S,V] in bf16. They are divided by T in place (bf16) and read twice, once by
// logprobs_from_logits (torch_utils.py:115-177) and once by chunked_entropy_from_logits
// (:59-111). The backward writes bf16 dlogits [n,S,V], which the lm_head backward GEMMs read.
//
// Here the vocabulary is cut into chunks of vc columns. For each chunk the host runs one plain
// library GEMM, Z_c = h @ W_c^T (hipBLASLt), into ONE reused bf16 [T,vc] buffer (about the
// size of the 256 MiB Infinity Cache). The kernels below consume it right after the GEMM:
//   forward : merge each chunk's rows into a per-token online-softmax state (m, S, W, x_label)
//             in log2 units, the same state as logprob.hip. The last chunk's launch finalizes
//             logp = x_label - lse, H = ln S - ln2 * W/S and lse. One wave per token row.
//   backward: dZ_c = (g_lp*(1[v=label] - p) - g_ent*p*(logp_v + H)) / T in bf16, into a reused
//             chunk buffer. The host then runs dH += dZ_c @ W_c (fp32 accumulate) and
//             dW_c = dZ_c^T @ h.
// The per-element numerics (bf16 division by T, exp2/log2 forms) equal logprob.hip's, so a
// chunked run equals the unfused kernels on the same bf16 logits up to the chunk-merge rounding.
#include "softmax.h"

namespace skyrl {
namespace {

constexpr int kThreads = 256;
constexpr int kRowsPerBlock = kThreads / kWave;
constexpr int kUnroll = 4;

// Per-token running state between chunk launches: m, S, W (log2 units) and the label logit.
struct __align__(16) ChunkState {
    float m, s, w, xl;
};

__global__ __launch_bounds__(kThreads) void lmhead_fwd_kernel(
    const uint16_t* __restrict__ z, int64_t ldz, int T, int vc, int64_t v0, const int64_t* __restrict__ labels,
    int64_t lstride, float temp, bool has_t, ChunkState* __restrict__ state, int first, int last,
    float* __restrict__ logp_out, float* __restrict__ ent_out, float* __restrict__ lse_out) {
    using E = Elem<uint16_t>;
    constexpr int VEC = E::kVec;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
    if (r >= T) return;
    const uint16_t* row = z + r * ldz;

    SoftState st;
    state_init(st);
    int done = 0;
    if ((reinterpret_cast<uintptr_t>(row) & 15) == 0) {
        // default-policy loads: the chunk was just written by the GEMM (partly L2/MALL-resident)
        const int nvec = vc / VEC;
        const uint4* rv = reinterpret_cast<const uint4*>(row);
        int i = lane;
        for (; i + (kUnroll - 1) * kWave < nvec; i += kUnroll * kWave) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) v[u] = rv[i + u * kWave];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                float x[VEC];
                E::unpack(v[u], x);
                if (has_t) {
#pragma unroll
                    for (int k = 0; k < VEC; ++k) x[k] = E::apply_t(x[k], temp, true);
                }
                state_add<VEC>(st, x);
            }
        }
        for (; i < nvec; i += kWave) {
            float x[VEC];
            E::unpack(rv[i], x);
            if (has_t) {
#pragma unroll
                for (int k = 0; k < VEC; ++k) x[k] = E::apply_t(x[k], temp, true);
            }
            state_add<VEC>(st, x);
        }
        done = nvec * VEC;
    }
    for (int i = done + lane; i < vc; i += kWave) {
        float x[1] = {E::apply_t(E::load(row + i), temp, has_t)};
        state_add<1>(st, x);
    }
    st = wave_merge(st);
    if (lane != 0) return;
    float xl = __builtin_nanf("");
    if (!first) {
        const ChunkState prev = state[r];
        SoftState ps{prev.m, prev.s, prev.w};
        state_merge(st, ps);
        xl = prev.xl;
    }
    const int64_t lab = labels[r * lstride];
    if (lab >= v0 && lab < v0 + vc) xl = E::apply_t(E::load(row + (lab - v0)), temp, has_t);
    if (!last) {
        state[r] = ChunkState{st.m, st.s, st.w, xl};
        return;
    }
    finalize_row(st, xl, r, logp_out, ent_out, lse_out);
}

__global__ __launch_bounds__(kThreads) void lmhead_bwd_kernel(
    const uint16_t* __restrict__ z, int64_t ldz, int T, int vc, int64_t v0, const int64_t* __restrict__ labels,
    int64_t lstride, float temp, bool has_t, const float* __restrict__ lse, const float* __restrict__ ent,
    const float* __restrict__ g_lp, const float* __restrict__ g_ent, uint16_t* __restrict__ dz, int64_t lddz) {
    using E = Elem<uint16_t>;
    constexpr int VEC = E::kVec;
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t r = (int64_t)blockIdx.x * kRowsPerBlock + threadIdx.x / kWave;
    if (r >= T) return;
    const uint16_t* row = z + r * ldz;
    uint16_t* out = dz + r * lddz;
    const float L = lse[r];
    const float H = g_ent ? ent[r] : 0.f;
    const float glp = g_lp[r];
    const float gent = g_ent ? g_ent[r] : 0.f;
    const float inv_t = has_t ? 1.f / temp : 1.f;
    const int64_t lab = labels[r * lstride] - v0;  // chunk-local label column
    auto grad = [&](float x, int64_t v) -> float {
        const float lp = x - L;
        const float p = fast_exp2(lp * kLog2e);
        float g = -glp * p - gent * p * (lp + H);
        if (v == lab) g += glp;
        return has_t ? g * inv_t : g;
    };
    int done = 0;
    if ((reinterpret_cast<uintptr_t>(row) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
        const int nvec = vc / VEC;
        const uint4* rv = reinterpret_cast<const uint4*>(row);
        uint4* ov = reinterpret_cast<uint4*>(out);
        int i = lane;
        for (; i + (kUnroll - 1) * kWave < nvec; i += kUnroll * kWave) {
            uint4 v[kUnroll];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) v[u] = rv[i + u * kWave];
#pragma unroll
            for (int u = 0; u < kUnroll; ++u) {
                float x[VEC];
                E::unpack(v[u], x);
                const int64_t c0 = (int64_t)(i + u * kWave) * VEC;
#pragma unroll
                for (int k = 0; k < VEC; ++k) x[k] = grad(E::apply_t(x[k], temp, has_t), c0 + k);
                ov[i + u * kWave] = E::pack(x);
            }
        }
        for (; i < nvec; i += kWave) {
            float x[VEC];
            E::unpack(rv[i], x);
            const int64_t c0 = (int64_t)i * VEC;
#pragma unroll
            for (int k = 0; k < VEC; ++k) x[k] = grad(E::apply_t(x[k], temp, has_t), c0 + k);
            ov[i] = E::pack(x);
        }
        done = nvec * VEC;
    }
    for (int i = done + lane; i < vc; i += kWave) E::store(out + i, grad(E::apply_t(E::load(row + i), temp, has_t), i));
}

// Vocab-parallel merge (DistributedLogprob, megatron/model_utils.py:26-136 + _VocabParallelEntropy
// :548-578): each tensor-parallel rank ran the chunk kernel over its vocab shard with last=0 and
// the ranks all-gathered the [T] states. One thread per token merges the nstates states (the
// label logit comes from the one shard holding the label) and finalizes like the last chunk.
__global__ __launch_bounds__(kThreads) void lmhead_state_merge_kernel(const ChunkState* __restrict__ states,
                                                                      int nstates, int T, float* __restrict__ logp_out,
                                                                      float* __restrict__ ent_out,
                                                                      float* __restrict__ lse_out) {
    const int64_t r = (int64_t)blockIdx.x * kThreads + threadIdx.x;
    if (r >= T) return;
    const ChunkState c0 = states[r];
    SoftState st{c0.m, c0.s, c0.w};
    float xl = c0.xl;
    for (int k = 1; k < nstates; ++k) {
        const ChunkState c = states[(int64_t)k * T + r];
        state_merge(st, SoftState{c.m, c.s, c.w});
        if (__builtin_isnan(xl)) xl = c.xl;
    }
    finalize_row(st, xl, r, logp_out, ent_out, lse_out);
}

inline unsigned blocks_for(int T) { return (unsigned)((T + kRowsPerBlock - 1) / kRowsPerBlock); }

}  // namespace
}  // namespace skyrl

using namespace skyrl;

extern "C" size_t skyrl_lmhead_state_bytes(int32_t T) { return (size_t)(T > 0 ? T : 1) * sizeof(ChunkState); }

extern "C" int skyrl_lmhead_chunk_fwd(const void* z, int64_t ldz, int32_t T, int32_t vc, int64_t v0,
                                      const int64_t* labels, int64_t label_stride, float temperature, void* state,
                                      int32_t first, int32_t last, float* logp_out, float* entropy_out,
                                      float* lse_out, void* stream) {
    SKYRL_REQUIRE(T >= 0 && vc > 0 && ldz >= vc && v0 >= 0, "lmhead_chunk_fwd: bad sizes");
    if (T == 0) return SKYRL_OK;
    SKYRL_REQUIRE(z && labels, "lmhead_chunk_fwd: null pointer");
    SKYRL_REQUIRE(temperature > 0.f, "lmhead_chunk_fwd: temperature must be > 0");
    SKYRL_REQUIRE(state || (first && last), "lmhead_chunk_fwd: state needed unless one chunk covers V");
    SKYRL_REQUIRE(!last || logp_out, "lmhead_chunk_fwd: logp_out needed on the last chunk");
    hipLaunchKernelGGL(lmhead_fwd_kernel, dim3(blocks_for(T)), dim3(kThreads), 0, as_stream(stream),
                       reinterpret_cast<const uint16_t*>(z), ldz, T, vc, v0, labels, label_stride, temperature,
                       temperature != 1.0f, reinterpret_cast<ChunkState*>(state), first != 0, last != 0, logp_out,
                       entropy_out, lse_out);
    return check_launch("lmhead_fwd_kernel");
}

extern "C" int skyrl_lmhead_chunk_bwd(const void* z, int64_t ldz, int32_t T, int32_t vc, int64_t v0,
                                      const int64_t* labels, int64_t label_stride, float temperature, const float* lse,
                                      const float* entropy, const float* grad_logp, const float* grad_entropy,
                                      void* dz, int64_t lddz, void* stream) {
    SKYRL_REQUIRE(T >= 0 && vc > 0 && ldz >= vc && lddz >= vc && v0 >= 0, "lmhead_chunk_bwd: bad sizes");
    if (T == 0) return SKYRL_OK;
    SKYRL_REQUIRE(z && labels && lse && grad_logp && dz, "lmhead_chunk_bwd: null pointer");
    SKYRL_REQUIRE(!grad_entropy || entropy, "lmhead_chunk_bwd: grad_entropy needs entropy");
    SKYRL_REQUIRE(temperature > 0.f, "lmhead_chunk_bwd: temperature must be > 0");
    hipLaunchKernelGGL(lmhead_bwd_kernel, dim3(blocks_for(T)), dim3(kThreads), 0, as_stream(stream),
                       reinterpret_cast<const uint16_t*>(z), ldz, T, vc, v0, labels, label_stride, temperature,
                       temperature != 1.0f, lse, entropy, grad_logp, grad_entropy, reinterpret_cast<uint16_t*>(dz),
                       lddz);
    return check_launch("lmhead_bwd_kernel");
}

extern "C" int skyrl_lmhead_state_merge(const void* states, int32_t nstates, int32_t T, float* logp_out,
                                        float* entropy_out, float* lse_out, void* stream) {
    SKYRL_REQUIRE(T >= 0 && nstates >= 1, "lmhead_state_merge: bad sizes");
    if (T == 0) return SKYRL_OK;
    SKYRL_REQUIRE(states && logp_out, "lmhead_state_merge: null pointer");
    hipLaunchKernelGGL(lmhead_state_merge_kernel, dim3((unsigned)((T + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       as_stream(stream), reinterpret_cast<const ChunkState*>(states), nstates, T, logp_out,
                       entropy_out, lse_out);
    return check_launch("lmhead_state_merge_kernel");
}
