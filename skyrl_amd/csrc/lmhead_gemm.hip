// SURVEY §8(f)1, decode side: the lm_head GEMM with the sampler fused into its epilogue, so the
// [n, V] decode logits never reach HBM.
//
// Reference: the rollout step's logits + sampler (vLLM's LogitsProcessor + Sampler behind
// VLLMInferenceEngine.generate, skyrl-train/skyrl_train/inference_engines/vllm/vllm_engine.py:
// 139-149,196-218; sampling params inference_engines/utils.py:15-42). The unfused path here is
// a library GEMM writing bf16 logits [n, V] followed by skyrl_sample (sampler.hip), which reads
// them back: 2 x 2 V bytes per row of HBM traffic on top of the GEMM.
//
// GEMM: Z = H W^T with H [M, K] (final-norm hidden states) and W [V, K] (the HF lm_head weight,
// both K-contiguous), bf16 in, fp32 accumulate on MFMA (v_mfma_f32_16x16x32_bf16).
//   * Tile 256 x 256 x 64 per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 outputs
//     per wave: 8 x 4 accumulators of 16 x 16). One workgroup per CU (128 KB of LDS).
//   * Operands stream HBM -> LDS with global_load_lds (16 B per lane, no VGPR round trip) into
//     two 64 KB stages; tile t+1 is in flight while tile t feeds the MFMAs. One barrier per K
//     step. LDS rows are 128 B, with the 16-B chunk index XOR-swizzled by (row >> 1) & 7 (the
//     swizzle is applied to the per-lane global source address, the LDS image stays
//     lane-linear) so the fragment reads (ds_read_b128, 16 rows x 4 chunks) are conflict-free.
//   * XCD-aware order: workgroup ids are remapped (bijectively) so that each XCD walks a
//     contiguous range of tiles with M fastest: the M tiles that share a W tile run together on
//     one XCD and read it once from HBM into that XCD's L2.
// Epilogue: the 256 x 256 accumulator tile is rounded to bf16 (the logits the unfused path
// would have written) into a swizzled LDS image, then
//   * STORE: written out as bf16 Z (the plain GEMM; also the parity handle for the fused path);
//   * SAMPLE / GREEDY: two threads per row run the sampler's decision (noise.h: group-of-8
//     exponential race, group bound, exact det_ln scores; greedy = first maximum) and the raw
//     online (max, sum-exp) over the tile's 256 columns. One 20-B partial per (row, tile).
// A one-wave-per-row merge folds a row's tile partials (argmax, lowest index on ties; LSE) into
// the token and its logprob log_softmax(raw logits)[token]. Decisions equal skyrl_sample's /
// oracle/sampler_ref.c's on the bf16 logits this GEMM produces (STORE), bit for bit.
#include "noise.h"
#include "softmax.h"
#include "variant.h"

namespace skyrl {
namespace {

constexpr int BM = 256;
constexpr float kLog2eG = 1.4426950408889634f;
constexpr float kLn2G = 0.6931471805599453f;

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) void gbl_void;
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

enum { EPI_STORE = 0, EPI_SAMPLE = 1, EPI_GREEDY = 2, EPI_LOGPROB = 3, EPI_LOGPROB_NOENT = 4 };

// Tile geometry: BM (256) x BN output columns, NT = 2 BN threads as 2 (M) x BN/64 (N) waves of
// 128 x 64 outputs; K in BKT-deep tiles through S LDS stages (S - 1 tiles in flight).
template <int BN, int BKT, int S, int NTH = 2 * BN>
struct Geo {
    static constexpr int NT = NTH;
    static constexpr int kWaves = NT / 64;
    static constexpr int kRowBytes = BKT * 2;                  // one operand row of a K tile
    static constexpr int kChunks = kRowBytes / 16;             // 16-B chunks per operand row
    static constexpr int kRowsPerWin = 256 / kRowBytes;        // operand rows per 256-B LDS bank window
    static constexpr int kOpABytes = BM * kRowBytes;           // H tile
    static constexpr int kStageBytes = (BM + BN) * kRowBytes;  // H tile + W tile
    static constexpr int kRowsPerPiece = 1024 / kRowBytes;     // rows per 1-KB wave copy (64 x 16 B)
    static constexpr int kPieces = (BM + BN) / kRowsPerPiece / kWaves;  // copies per wave per stage
    static constexpr int KS = BKT / 32;                        // 16x16x32 k-steps per K tile
    // epilogue image [BM][BN] bf16; TPR threads per row, thread hh of a row owns chunks TPR i + hh
    static constexpr int kImgRow = BN * 2;
    static constexpr int kImgBytes = BM * kImgRow;
    static constexpr int kCpr = BN / 8;
    static constexpr int TPR = NT / BM;
    static constexpr int kChunksPerThread = kCpr / TPR;
    static constexpr int kLds = S * kStageBytes > kImgBytes ? S * kStageBytes : kImgBytes;
    static_assert(S >= 2 && kLds <= 160 * 1024, "LDS");
    static_assert((BM + BN) % (kRowsPerPiece * kWaves) == 0, "staging split");
    // operand chunk swizzle: the 16 rows of a fragment read hit 16 distinct 16-B bank slots
    __device__ static int swz(int row) { return (row / kRowsPerWin) % kChunks; }
    // image chunk swizzle: a 16-lane read group (16 / TPR rows x TPR parities) is conflict-free
    __device__ static int img_off(int r, int c) { return r * kImgRow + ((c ^ ((r & (16 / TPR - 1)) * TPR)) << 4); }
};

// Cross-tile row bar of the sampling epilogue: the best exact score any finished tile of the row
// found, as an order-preserving 32-bit key (atomic max in global memory); 0 = none yet (also the
// zeroed workspace and what the merge kernel re-arms it to).
__device__ __forceinline__ unsigned bar_key(float sc) {
    const uint32_t u = __float_as_uint(sc + 0.0f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float bar_value(unsigned k) {
    if (k <= 0x007fffffu) return -INFINITY;  // none yet (or -inf)
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}
// hardware natural log (v_log_f32 is log2): within ~3e-6 of det_ln for the arguments here
__device__ __forceinline__ float hw_ln(float x) { return __builtin_amdgcn_logf(x) * kLn2G; }
// the group bound's slope in score units: ln2 2^-23 per unit of bits(float(h16)) (noise.h)
constexpr float kBitsLn2 = 0.6931471805599453f * 1.1920928955078125e-7f;

template <int N>
__device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// the variant field lmhead_pipe selects the K pipeline (pick_kernel): 0 = 256 x 256 tiles, BK 64, 2
// stages, one 512-thread workgroup per CU; 1 = 256 x 128 tiles, BK 32, 3 stages, two workgroups
// per CU; 2 = 256 x 256, BK 32, 4 stages; 3-10 = staggered copies / fragment double buffer /
// spread copies; 11 = ping-pong wave groups (4 phases per K step); 12 (default) = the fragment
// double buffer of 4 with three W stages and two H stages. All produce identical Z. Measured
// (profiles/r02_gemm_*): 12 is the fastest at 512, 2048 and 8192 rows; 11 is slower
// even without copies (8 barriers per K step).

// scripts/probe/gemm_noload.py only (never in the product build): the K loop re-reads the
// prologue's tiles instead of copying new ones, to time the loop structure without memory.
#ifdef SKYRL_GEMM_NOLOAD
constexpr bool kNoLoad = true;
#else
constexpr bool kNoLoad = false;
#endif
// probe-only: drop only the H (NOLOAD_H) or only the W (NOLOAD_W) copies of pipe 12's K loop
#ifdef SKYRL_GEMM_NOLOAD_H
constexpr bool kNoLoadH = true;
#else
constexpr bool kNoLoadH = kNoLoad;
#endif
#ifdef SKYRL_GEMM_NOLOAD_W
constexpr bool kNoLoadW = true;
#else
constexpr bool kNoLoadW = kNoLoad;
#endif

// Phase timestamps for scripts/probe/lmhead_phase_probe (compiled only there, never in the product).
#ifdef SKYRL_GEMM_PHASE_PROBE
__device__ uint64_t g_gphase[4096 * 8];
#define GPHASE(k)                                                                   \
    do {                                                                            \
        if (threadIdx.x == 0 && blockIdx.x < 4096)                                  \
            g_gphase[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime();      \
    } while (0)
#else
#define GPHASE(k) \
    do {          \
    } while (0)
#endif

// DB 6 runs 4 waves of 128 x 128 outputs (one per SIMD, accumulators in AGPRs); the others run
// 2 BN threads, two waves per SIMD.
template <int EPI, int BN, int BKT, int S, int STAGGER, int DB>
__global__ __launch_bounds__(DB == 6 ? 256 : 2 * BN) __attribute__((amdgpu_waves_per_eu(DB == 6 ? 1 : 2))) void lmhead_gemm_kernel(
    const uint16_t* __restrict__ H, int64_t ldh, const uint16_t* __restrict__ W, int64_t ldw, int M, int N, int K,
    int mtg, uint16_t* __restrict__ Z, int64_t ldz, float inv_t, uint64_t seed, const int64_t* __restrict__ seq_ids,
    int64_t step, float4* __restrict__ parts, float* __restrict__ part_x, int nt, const int64_t* __restrict__ labels,
    int64_t lstride, unsigned* __restrict__ rowbar) {
    using G = Geo<BN, BKT, S, DB == 6 ? 256 : 2 * BN>;
    constexpr int NB = DB == 6 ? 8 : 4;  // 16-column accumulator tiles per wave
    // DB 5 and 6 keep two H stages and three W stages: the whole 160 KB
    __shared__ __attribute__((aligned(16))) char smem[DB == 5 || DB == 6 ? 163840 : G::kLds];
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    // tile order: mtg = mt | gm << 16. gm = 0: M fastest over all M tiles (the M tiles sharing a W
    // tile run together); gm > 0: groups of gm M tiles, M fastest inside a group, so an XCD's
    // concurrent tiles share gm H tiles that stay L2-resident across the W tiles it walks
    GPHASE(0);
    const int mt = mtg & 0xffff, gm = mtg >> 16;
    int mtile, ntile;
    if (gm <= 0 || gm >= mt) {
        mtile = wg % mt;
        ntile = wg / mt;
    } else {
        const int per = gm * nt, gi = wg / per, r = wg - gi * per, gsz = min(gm, mt - gi * gm);
        mtile = gi * gm + r % gsz;
        ntile = r / gsz;
    }
    const int m0 = mtile * BM, n0 = ntile * BN;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // DB 4 (ping-pong): wave group wm = w >> 2 holds one wave of each SIMD; otherwise wm = w & 1
    // (DB 6: 2 x 2 waves of 128 x 128)
    const int wm = DB == 4 ? (w >> 2) : (w & 1), wn = DB == 4 ? (w & 3) : (w >> 1);

    f32x4 acc[8][NB];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    if constexpr (DB == 7) {
        // W fragments straight from global memory into registers (no LDS write or read for W), H
        // through two LDS stages with global_load_lds. Step t's W fragments are loaded at the top of
        // step t - 1 into the other register buffer; each row's 128 B of a K step are read as two
        // 64-B halves by the 16-lane groups (ks = 0, 1), and the two waves of a wave column read the
        // same fragments (the second from L1).
        static_assert(BN == 256 && BKT == 64 && S == 2, "W-in-registers geometry");
        constexpr int kT = 32768, kRow = 128;
        const uint16_t* hs[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = (w * 4 + j) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ G::swz(row);
            hs[j] = H + (int64_t)min(m0 + row, M - 1) * ldh + c * 8;
        }
        char* const hdst = smem + w * 4 * 1024;
        auto copyH = [&](int tile) {
            if (kNoLoad && tile >= 1) return;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(hs[j] + tile * 64),
                                                 (lds_void*)(hdst + (tile & 1) * kT + j * 1024), 16, 0, 0);
        };
        const uint16_t* wrow[4];  // this lane's W row of each 16-column fragment, at its k offset
#pragma unroll
        for (int nb = 0; nb < 4; ++nb)
            wrow[nb] = W + (int64_t)min(n0 + wn * 64 + nb * 16 + (lane & 15), N - 1) * ldw + (lane >> 4) * 8;
        bf16x8 bw[2][2][4];  // [buffer][ks][nb]
        auto loadW = [&](int buf, int tile) {
            if (kNoLoad && tile >= 1) return;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
                    bw[buf][ks][nb] = *reinterpret_cast<const bf16x8*>(wrow[nb] + tile * 64 + ks * 32);
        };
        int aoff[2];
        {
            const int sw = G::swz(lane & 15);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) aoff[ks] = (wm * 128 + (lane & 15)) * kRow + (((ks * 4 + (lane >> 4)) ^ sw) * 16);
        }
        const int nk = K / 64;
        copyH(0);
        loadW(0, 0);
        // one K step with the W fragments in register buffer CB (compile-time: no selects)
        auto kstep = [&](int t, auto cb_tag) {
            constexpr int CB = decltype(cb_tag)::value;
            wait_vmcnt<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            const char* sa = smem + (t & 1) * kT;
            if (t + 1 < nk) {
                copyH(t + 1);
                loadW(1 - CB, t + 1);
            }
            bf16x8 aq[2][2];
            auto ldA = [&](int ks, int mp, bf16x8 (&dst)[2]) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    dst[u] = *reinterpret_cast<const bf16x8*>(sa + aoff[ks] + (2 * mp + u) * 16 * kRow);
            };
            ldA(0, 0, aq[0]);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const int ks = g / 4, mp = g % 4;
                if (g + 1 < 8) ldA((g + 1) / 4, (g + 1) % 4, aq[(g + 1) & 1]);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        acc[2 * mp + u][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            aq[g & 1][u], bw[CB][ks][nb], acc[2 * mp + u][nb], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        for (int t = 0; t < nk; t += 2) {
            kstep(t, std::integral_constant<int, 0>{});
            if (t + 1 < nk) kstep(t + 1, std::integral_constant<int, 1>{});
        }
    } else if constexpr (DB == 6) {
        // Four waves, 128 x 128 outputs each (8 x 8 accumulators): per MFMA a wave reads 2/3 of
        // the LDS bytes of the 128 x 64 layout (A and B fragments reused 8 times instead of 4 and
        // 8), which matters because the glds writes share the LDS with the fragment reads.
        // Staging as DB 5 (three W stages, two H stages); each wave copies 8 H and 8 W pieces.
        static_assert(BN == 256 && BKT == 64 && S == 2, "4-wave geometry");
        constexpr int kT = 32768, kWBase = 2 * kT, kRow = 128;
        // piece j of wave w covers operand rows w*64 + 8j .. + 7; lane -> row + lane / 8, chunk
        // lane & 7 (the chunk swizzle (row >> 1) & 7 alternates with j's parity)
        const int brow = w * 64 + (lane >> 3);
        // 32-bit element offsets (the host picks this pipeline only when M ldh and N ldw < 2^31)
        uint32_t hoff[8], woff[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int row = brow + 8 * j;
            const int c = (lane & 7) ^ G::swz(row);
            hoff[j] = (uint32_t)min(m0 + row, M - 1) * (uint32_t)ldh + c * 8;
            woff[j] = (uint32_t)min(n0 + row, N - 1) * (uint32_t)ldw + c * 8;
        }
        char* const hdst = smem + w * 8 * 1024;
        char* const wdst = smem + kWBase + w * 8 * 1024;
        auto copyH = [&](int tile) {
            if (kNoLoad && tile >= 1) return;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(H + hoff[j] + tile * 64),
                                                 (lds_void*)(hdst + (tile & 1) * kT + j * 1024), 16, 0, 0);
        };
        auto copyW = [&](int tile) {
            if (kNoLoad && tile >= 2) return;
#pragma unroll
            for (int j = 0; j < 8; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(W + woff[j] + tile * 64),
                                                 (lds_void*)(wdst + (tile % 3) * kT + j * 1024), 16, 0, 0);
        };
        int aoff[2], boff[2];
        {
            const int sw = G::swz(lane & 15);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int c = (ks * 4 + (lane >> 4)) ^ sw;
                aoff[ks] = (wm * 128 + (lane & 15)) * kRow + c * 16;
                boff[ks] = kWBase + (wn * 128 + (lane & 15)) * kRow + c * 16;
            }
        }
        const int nk = K / 64;
        copyH(0);
        copyW(0);
        if (nk > 1) copyW(1);
        for (int t = 0; t < nk; ++t) {
            if (t + 1 < nk) wait_vmcnt<8>();
            else wait_vmcnt<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            const char* sa = smem + (t & 1) * kT;
            const char* sbw = smem + (t % 3) * kT;  // + boff's kWBase
            if (t + 1 < nk) copyH(t + 1);
            if (t + 2 < nk) copyW(t + 2);
            // groups of 2 A fragments x 8 B fragments (16 MFMAs); the next group's ds_reads (and
            // the next k-step's 8 B fragments) are issued before this group's MFMAs
            bf16x8 bq[2][8], aq[2][2];
            auto ldA = [&](int ks, int mp, bf16x8 (&dst)[2]) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    dst[u] = *reinterpret_cast<const bf16x8*>(sa + aoff[ks] + (2 * mp + u) * 16 * kRow);
            };
            auto ldB = [&](int ks) {
#pragma unroll
                for (int nb = 0; nb < 8; ++nb)
                    bq[ks][nb] = *reinterpret_cast<const bf16x8*>(sbw + boff[ks] + nb * 16 * kRow);
            };
            ldB(0);
            ldA(0, 0, aq[0]);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const int ks = g / 4, mp = g % 4;
                if (g + 1 < 8) {
                    if ((g + 1) % 4 == 0) ldB((g + 1) / 4);
                    ldA((g + 1) / 4, (g + 1) % 4, aq[(g + 1) & 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int nb = 0; nb < 8; ++nb)
                        acc[2 * mp + u][nb] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[g & 1][u], bq[ks][nb], acc[2 * mp + u][nb], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else if constexpr (DB == 5) {
        // Asymmetric stages: the W tile of K step t + 2 and the H tile of step t + 1 are in flight
        // while step t computes. At the decode shape H (a few hundred rows) is L2-resident and W
        // streams from HBM once, so the slow operand gets two steps of latency cover. LDS: H
        // stages at [0, 64 KB), W stages at [64 KB, 160 KB), 256 rows x 128 B each, the 16-B
        // chunk swizzle of Geo. Every wave copies 4 H and 4 W pieces per step, H first, so at the
        // top of step t only W(t + 1)'s 4 copies may stay outstanding.
        static_assert(BN == 256 && BKT == 64 && S == 2, "asymmetric-stage geometry");
        constexpr int kT = 32768, kWBase = 2 * kT, kRow = 128;
        const uint16_t* hs[4];
        const uint16_t* wsrc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int row = (w * 4 + j) * 8 + (lane >> 3);
            const int c = (lane & 7) ^ G::swz(row);
            hs[j] = H + (int64_t)min(m0 + row, M - 1) * ldh + c * 8;
            wsrc[j] = W + (int64_t)min(n0 + row, N - 1) * ldw + c * 8;
        }
        char* const hdst = smem + w * 4 * 1024;
        char* const wdst = smem + kWBase + w * 4 * 1024;
        auto copyH = [&](int tile) {
            if (kNoLoadH && tile >= 1) return;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(hs[j] + tile * 64),
                                                 (lds_void*)(hdst + (tile & 1) * kT + j * 1024), 16, 0, 0);
        };
        auto copyW = [&](int tile) {
            if (kNoLoadW && tile >= 2) return;
#pragma unroll
            for (int j = 0; j < 4; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(wsrc[j] + tile * 64),
                                                 (lds_void*)(wdst + (tile % 3) * kT + j * 1024), 16, 0, 0);
        };
        int aoff[2], boff[2];
        {
            const int sw = G::swz(lane & 15);
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const int c = (ks * 4 + (lane >> 4)) ^ sw;
                aoff[ks] = (wm * 128 + (lane & 15)) * kRow + c * 16;
                boff[ks] = kWBase + (wn * 64 + (lane & 15)) * kRow + c * 16;
            }
        }
        const int nk = K / 64;
        copyH(0);
        copyW(0);
        if (nk > 1) copyW(1);
        for (int t = 0; t < nk; ++t) {
            if (t + 1 < nk) wait_vmcnt<4>();
            else wait_vmcnt<0>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            const char* sa = smem + (t & 1) * kT;
            const char* sbw = smem + (t % 3) * kT;  // + boff's kWBase
            if (t + 1 < nk) copyH(t + 1);
            if (t + 2 < nk) copyW(t + 2);
            // fragment pipeline of DB 1: groups of 2 A x 4 B fragments (8 MFMAs), the next group's
            // ds_reads issued before this group's MFMAs
            bf16x8 bq[2][4], aq[2][2];
            auto ldA = [&](int ks, int mp, bf16x8 (&dst)[2]) {
#pragma unroll
                for (int u = 0; u < 2; ++u)
                    dst[u] = *reinterpret_cast<const bf16x8*>(sa + aoff[ks] + (2 * mp + u) * 16 * kRow);
            };
            auto ldB = [&](int ks) {
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
                    bq[ks][nb] = *reinterpret_cast<const bf16x8*>(sbw + boff[ks] + nb * 16 * kRow);
            };
            ldB(0);
            ldA(0, 0, aq[0]);
#pragma unroll
            for (int g = 0; g < 8; ++g) {
                const int ks = g / 4, mp = g % 4;
                if (g + 1 < 8) {
                    if ((g + 1) % 4 == 0) ldB((g + 1) / 4);
                    ldA((g + 1) / 4, (g + 1) % 4, aq[(g + 1) & 1]);
                }
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int u = 0; u < 2; ++u)
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        acc[2 * mp + u][nb] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[g & 1][u], bq[ks][nb], acc[2 * mp + u][nb], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    } else if constexpr (DB == 4) {
        // Ping-pong schedule. The K tile's LDS buffer holds four 16-KB operand halves: A0 / A1 are
        // the H rows of output-quadrant row 0 / 1 of both wave groups (group g's rows g*128 + q*64
        // + r), B0 / B1 the W rows of quadrant column 0 / 1 of the four wave columns (wn*64 + q*32
        // + r). A tile runs as four phases, one 64 x 32 output quadrant of every wave per phase
        // ((0,0), (0,1), (1,1), (1,0): A0+B0, B1, A1, B0 fragment reads), each phase a load
        // interval (fragment reads, one half-tile copy, counted vmcnt, lgkmcnt(0)), s_barrier,
        // 16 MFMAs, s_barrier. Group 1 runs one barrier behind group 0, so on every SIMD one
        // wave's MFMAs overlap the other wave's loads.
        // Copies: phase 0 of tile t stages B0 of t + 1, phase 1 A1 of t + 1, phase 2 A0 of t + 2,
        // phase 3 B1 of t + 2 -- each one phase after the last read of the half it overwrites (the
        // reads were retired by lgkmcnt(0) before the barrier that ends their load interval), and
        // at least four phases before its first read. The wait after a phase's copy retires the
        // copies of three phases earlier and older (vmcnt <= 6), so a half staged at phase f is
        // complete in every wave before the barrier that precedes the reads of phase f + 4.
        static_assert(BN == 256 && BKT == 64 && S == 2, "ping-pong geometry");
        constexpr int kHalf = 16384, kBuf = 4 * kHalf, kRow = 128;
        const uint16_t* src[4][2];
#pragma unroll
        for (int h = 0; h < 4; ++h)
#pragma unroll
            for (int j = 0; j < 2; ++j) {
                const int hr = (2 * w + j) * 8 + (lane >> 3);    // half row of this lane's 16 B
                const int c = (lane & 7) ^ ((hr >> 1) & 7);      // logical chunk landing in chunk lane & 7
                if (h < 2) {
                    const int grow = min(m0 + (hr >> 6) * 128 + h * 64 + (hr & 63), M - 1);
                    src[h][j] = H + (int64_t)grow * ldh + c * 8;
                } else {
                    const int grow = min(n0 + (hr >> 5) * 64 + (h - 2) * 32 + (hr & 31), N - 1);
                    src[h][j] = W + (int64_t)grow * ldw + c * 8;
                }
            }
        char* const cdst = smem + 2 * w * 1024;
        auto copy = [&](int h, int tile) {
            if (kNoLoad && tile >= 2) return;
#pragma unroll
            for (int j = 0; j < 2; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(src[h][j] + tile * 64),
                                                 (lds_void*)(cdst + (tile & 1) * kBuf + h * kHalf + j * 1024), 16, 0, 0);
        };
        int aoff[2], boff[2];
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = (ks * 4 + (lane >> 4)) ^ ((lane & 15) >> 1);
            aoff[ks] = (wm * 64 + (lane & 15)) * kRow + c * 16;
            boff[ks] = 2 * kHalf + (wn * 32 + (lane & 15)) * kRow + c * 16;
        }
        const int nk = K / 64;
        // copies issued by global phase f (0 or 1 half-tile)
        auto issued = [&](int f) -> int { return f >= 0 && ((f & 3) < 2 ? (f >> 2) + 1 : (f >> 2) + 2) < nk; };
        copy(0, 0);
        copy(2, 0);
        copy(3, 0);
        copy(1, 0);
        if (nk > 1) {
            copy(0, 1);
            copy(3, 1);
            wait_vmcnt<4>();
        } else {
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        if (wm == 1) __builtin_amdgcn_s_barrier();
        bf16x8 fa[2][4], fb[2][2];
        for (int t = 0; t < nk; ++t) {
            const char* sb = smem + (t & 1) * kBuf;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int qm = p >> 1, qn = (p == 1 || p == 2) ? 1 : 0;
                __builtin_amdgcn_sched_barrier(0);
                if (p != 2) {
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                        for (int nb = 0; nb < 2; ++nb)
                            fb[ks][nb] = *reinterpret_cast<const bf16x8*>(sb + qn * kHalf + boff[ks] + nb * 16 * kRow);
                }
                if (p == 0 || p == 2) {
#pragma unroll
                    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                        for (int mb = 0; mb < 4; ++mb)
                            fa[ks][mb] = *reinterpret_cast<const bf16x8*>(sb + qm * kHalf + aoff[ks] + mb * 16 * kRow);
                }
                const int f = 4 * t + p;
                const int tc = p < 2 ? t + 1 : t + 2;
                if (tc < nk) copy(p == 0 ? 2 : p == 1 ? 1 : p == 2 ? 0 : 3, tc);
                switch (issued(f) + issued(f - 1) + issued(f - 2)) {
                    case 0: wait_vmcnt<0>(); break;
                    case 1: wait_vmcnt<2>(); break;
                    case 2: wait_vmcnt<4>(); break;
                    default: wait_vmcnt<6>(); break;
                }
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_setprio(1);
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int mb = 0; mb < 4; ++mb)
#pragma unroll
                        for (int nb = 0; nb < 2; ++nb)
                            acc[4 * qm + mb][2 * qn + nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                fa[ks][mb], fb[ks][nb], acc[4 * qm + mb][2 * qn + nb], 0, 0, 0);
                __builtin_amdgcn_s_setprio(0);
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_barrier();
            }
        }
        if (wm == 0) __builtin_amdgcn_s_barrier();
    } else {
        // staging: the stage is (BM + BN) operand rows (H rows, then W rows), copied as 1-KB pieces;
        // wave w copies pieces w * kPieces + j (the piece's LDS offset is wave-uniform: p * 1 KB)
        const int lrow = lane / G::kChunks, pc = lane % G::kChunks;
        const uint16_t* gsrc[G::kPieces];
#pragma unroll
        for (int j = 0; j < G::kPieces; ++j) {
            const int row = (w * G::kPieces + j) * G::kRowsPerPiece + lrow;  // stage row
            const int c = pc ^ G::swz(row);  // the logical chunk that lands in physical chunk pc
            const bool isw = row >= BM;
            const int rloc = isw ? row - BM : row;
            const int grow = isw ? min(n0 + rloc, N - 1) : min(m0 + rloc, M - 1);
            gsrc[j] = (isw ? W + (int64_t)grow * ldw : H + (int64_t)grow * ldh) + c * 8;
        }
        char* const sdst = smem + w * G::kPieces * 1024;
        auto stage = [&](int buf, int k0) {
            if (kNoLoad && k0 >= (S - 1) * BKT) return;
#pragma unroll
            for (int j = 0; j < G::kPieces; ++j)
                __builtin_amdgcn_global_load_lds((gbl_void*)(gsrc[j] + k0),
                                                 (lds_void*)(sdst + buf * G::kStageBytes + j * 1024), 16, 0, 0);
        };
        // fragment offsets: rows wm*128 + mb*16 + (lane & 15) of H, wn*64 + nb*16 + (lane & 15) of W;
        // k chunk ks*4 + (lane >> 4) (16x16x32 operand map); the swizzle depends on lane & 15 only
        int aoff[G::KS], boff[G::KS];
        {
            const int sw = G::swz(lane & 15);
#pragma unroll
            for (int ks = 0; ks < G::KS; ++ks) {
                const int c = (ks * 4 + (lane >> 4)) ^ sw;
                aoff[ks] = (wm * 128 + (lane & 15)) * G::kRowBytes + c * 16;
                boff[ks] = G::kOpABytes + (wn * 64 + (lane & 15)) * G::kRowBytes + c * 16;
            }
        }

        const int nk = K / BKT;
#pragma unroll
        for (int p = 0; p < S - 1; ++p)
            if (p < nk) stage(p, p * BKT);
        for (int t = 0; t < nk; ++t) {
            // tile t has landed once at most min(S - 2, nk - 1 - t) younger tiles are outstanding;
            // every wave's fragment reads of the buffer restaged below are done (WAR), then the barrier
            const int ahead = min(S - 2, nk - 1 - t);
            if (ahead <= 0) wait_vmcnt<0>();
            else if (ahead == 1) wait_vmcnt<G::kPieces>();
            else wait_vmcnt<2 * G::kPieces>();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            const char* sb = smem + (t % S) * G::kStageBytes;
            // STAGGER: the waves of the upper half (the second wave of each SIMD) issue their copies
            // after the first half of the k-steps, so a SIMD's MFMA pipe is never idle for both waves'
            // copy issue at once
            const bool late = STAGGER && __builtin_amdgcn_readfirstlane(w) >= G::kWaves / 2;
            const bool more = t + S - 1 < nk;
            if (DB != 2 && !late && more) stage((t + S - 1) % S, (t + S - 1) * BKT);
            if constexpr (DB == 3) {
                // k-step granularity: all fragments of k-step ks + 1 are read while k-step ks's MFMAs run
                // (issued after its first 8 MFMAs, so the compiler's lgkmcnt(0) -- it never counts LDS
                // waits while an LDS DMA is in flight -- only waits for reads that had 24 MFMAs of time)
                bf16x8 bq[G::KS][4], aq[G::KS][8];
                auto ld = [&](int ks) {
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        bq[ks][nb] = *reinterpret_cast<const bf16x8*>(sb + boff[ks] + nb * 16 * G::kRowBytes);
#pragma unroll
                    for (int mb = 0; mb < 8; ++mb)
                        aq[ks][mb] = *reinterpret_cast<const bf16x8*>(sb + aoff[ks] + mb * 16 * G::kRowBytes);
                };
                ld(0);
#pragma unroll
                for (int ks = 0; ks < G::KS; ++ks) {
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int mb = 0; mb < 8; ++mb) {
                        if (mb == 2 && ks + 1 < G::KS) {
                            __builtin_amdgcn_sched_barrier(0);
                            ld(ks + 1);
                            __builtin_amdgcn_sched_barrier(0);
                        }
#pragma unroll
                        for (int nb = 0; nb < 4; ++nb)
                            acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[ks][mb], bq[ks][nb], acc[mb][nb], 0, 0, 0);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);
                continue;
            }
            if constexpr (DB) {
                // explicit fragment pipeline: groups of 2 A fragments x 4 B fragments (8 MFMAs); the next
                // group's ds_reads are issued before this group's MFMAs, and sched_barriers keep the
                // compiler from sinking them (left alone it waits lgkmcnt(0) before every 8 MFMAs)
                constexpr int NG = G::KS * 4;
                bf16x8 bq[G::KS][4], aq[2][2];
                auto ldA = [&](int ks, int mp, bf16x8 (&dst)[2]) {
#pragma unroll
                    for (int u = 0; u < 2; ++u)
                        dst[u] = *reinterpret_cast<const bf16x8*>(sb + aoff[ks] + (2 * mp + u) * 16 * G::kRowBytes);
                };
                auto ldB = [&](int ks) {
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        bq[ks][nb] = *reinterpret_cast<const bf16x8*>(sb + boff[ks] + nb * 16 * G::kRowBytes);
                };
                ldB(0);
                ldA(0, 0, aq[0]);
#pragma unroll
                for (int g = 0; g < NG; ++g) {
                    const int ks = g / 4, mp = g % 4;
                    if (late && g == NG / 2 && more) stage((t + S - 1) % S, (t + S - 1) * BKT);
                    if (DB == 2 && more) {  // copies spread over the groups, in the pinned prefetch slot
#pragma unroll
                        for (int j = 0; j < G::kPieces; ++j)
                            if (j * NG / G::kPieces == g)
                                __builtin_amdgcn_global_load_lds((gbl_void*)(gsrc[j] + (t + S - 1) * BKT),
                                                                 (lds_void*)(sdst + ((t + S - 1) % S) * G::kStageBytes + j * 1024),
                                                                 16, 0, 0);
                    }
                    if (g + 1 < NG) {
                        if ((g + 1) % 4 == 0) ldB((g + 1) / 4);
                        ldA((g + 1) / 4, (g + 1) % 4, aq[(g + 1) & 1]);
                    }
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int u = 0; u < 2; ++u)
#pragma unroll
                        for (int nb = 0; nb < 4; ++nb)
                            acc[2 * mp + u][nb] =
                                __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[g & 1][u], bq[ks][nb], acc[2 * mp + u][nb], 0, 0, 0);
                    __builtin_amdgcn_sched_barrier(0);
                }
                continue;
            }
#pragma unroll
            for (int ks = 0; ks < G::KS; ++ks) {
                if (late && ks == G::KS / 2 && t + S - 1 < nk) stage((t + S - 1) % S, (t + S - 1) * BKT);
                bf16x8 b[4];
#pragma unroll
                for (int nb = 0; nb < 4; ++nb) b[nb] = *reinterpret_cast<const bf16x8*>(sb + boff[ks] + nb * 16 * G::kRowBytes);
#pragma unroll
                for (int mb = 0; mb < 8; ++mb) {
                    const bf16x8 a = *reinterpret_cast<const bf16x8*>(sb + aoff[ks] + mb * 16 * G::kRowBytes);
#pragma unroll
                    for (int nb = 0; nb < 4; ++nb)
                        acc[mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[nb], acc[mb][nb], 0, 0, 0);
                }
            }
        }
    }
    // every wave's last fragment reads are done before the image overwrites the stages
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();

    GPHASE(1);
    // ---- epilogue: bf16 tile into the LDS image (C map: row (lane >> 4) * 4 + i, col lane & 15)
#pragma unroll
    for (int mb = 0; mb < 8; ++mb)
#pragma unroll
        for (int nb = 0; nb < NB; ++nb)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int r = wm * 128 + mb * 16 + (lane >> 4) * 4 + i;
                const int c = wn * (NB * 16) + nb * 16 + (lane & 15);
                *reinterpret_cast<uint16_t*>(smem + G::img_off(r, c >> 3) + (c & 7) * 2) = f32_to_bf16(acc[mb][nb][i]);
            }
    __syncthreads();
    GPHASE(2);

    if constexpr (EPI == EPI_STORE) {
        const bool vec = (ldz & 7) == 0 && (reinterpret_cast<uintptr_t>(Z) & 15) == 0;
        constexpr int kIters = BM * G::kCpr / G::NT;
#pragma unroll 4
        for (int it = 0; it < kIters; ++it) {
            const int lin = it * G::NT + threadIdx.x;
            const int r = lin / G::kCpr, c = lin % G::kCpr;
            const int grow = m0 + r, col = n0 + c * 8;
            if (grow >= M || col >= N) continue;
            const uint4 v = *reinterpret_cast<const uint4*>(smem + G::img_off(r, c));
            uint16_t* dst = Z + (int64_t)grow * ldz + col;
            if (vec && col + 8 <= N) {
                *reinterpret_cast<uint4*>(dst) = v;
            } else {
                uint16_t e[8];
                __builtin_memcpy(e, &v, 16);
                for (int k = 0; k < 8 && col + k < N; ++k) dst[k] = e[k];
            }
        }
        return;
    } else if constexpr (EPI == EPI_LOGPROB) {
        // learner forward (old / ref log-probs): the per-token online-softmax state of the tile's
        // columns (logprob.hip's state: m, S = sum 2^y, W = sum 2^y y in log2 units, after the
        // reference's bf16 division by T) and the label's logit when the label is in this tile;
        // state [ntile][M] for skyrl_lmhead_state_merge. inv_t carries T (> 0), seed != 0 = T != 1.
        using E = Elem<uint16_t>;
        const float temp = inv_t;
        const bool has_t = seed != 0ull;
        const int r = threadIdx.x / G::TPR, hh = threadIdx.x % G::TPR;
        const int grow = m0 + r;
        if (grow >= M) return;
        SoftState st;
        state_init(st);
#pragma unroll 4
        for (int i = 0; i < G::kChunksPerThread; ++i) {
            const int c = G::TPR * i + hh;
            const int v0 = n0 + c * 8;
            const int cnt = min(8, N - v0);
            if (cnt <= 0) break;
            const uint4 pk = *reinterpret_cast<const uint4*>(smem + G::img_off(r, c));
            float x[8];
            E::unpack(pk, x);
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = k < cnt ? E::apply_t(x[k], temp, has_t) : -INFINITY;
            state_add<8>(st, x);
        }
#pragma unroll
        for (int o = 1; o < G::TPR; o <<= 1) {
            SoftState ot;
            ot.m = __shfl_xor(st.m, o, kWave);
            ot.s = __shfl_xor(st.s, o, kWave);
            ot.w = __shfl_xor(st.w, o, kWave);
            state_merge(st, ot);
        }
        if (hh == 0) {
            const int64_t lab = labels[(int64_t)grow * lstride] - n0;
            float xl = __builtin_nanf("");
            if (lab >= 0 && lab < BN && n0 + lab < N)
                xl = E::apply_t(bf16_to_f32(*reinterpret_cast<const uint16_t*>(
                                    smem + G::img_off(r, (int)lab >> 3) + ((int)lab & 7) * 2)),
                                temp, has_t);
            parts[(int64_t)ntile * M + grow] = make_float4(st.m, st.s, st.w, xl);
        }
    } else {
        constexpr bool greedy = EPI == EPI_GREEDY;
        constexpr int TPR = G::TPR, NC = G::kChunksPerThread;
        const int r = threadIdx.x / TPR, hh = threadIdx.x % TPR;
        const int grow = m0 + r;
        if (grow >= M) return;  // the threads of a row leave together (the row shuffle below)
        uint4 pk[NC];
        float m = -1e30f, s = 0.f;   // raw online (max, sum-exp)
        float best_s = -INFINITY, best_x = -INFINITY;
        int best_i = 0x7fffffff;
        float ubc[NC], vmx[NC];      // per group: c_g >= -ln E_v + 0.01 for each of its slots; its max logit
        uint32_t hg[NC];             // per group: its hash
        float best_ub = -INFINITY;   // pass 1: the best group bound (its first maximum and its
        int seed_g = -1, seed_k = 0; // minimum-E slot seed the bar)
        uint32_t key = 0u, key2 = 0u, keyb = 0u;
        if constexpr (!greedy) {
            key = row_key(seed, seq_ids ? seq_ids[grow] : (int64_t)grow, step);
            key2 = noise_key2(key);
            keyb = noise_keyb(key);
        }
        // pass 1, every group: LSE; greedy: the first maximum; sampling: the group bound of the
        // sampler kernels (one hash, no logarithm: E_v >= E_g > h16 2^-19, so -ln E_v <
        // ln2 (146 - bits(float(h16)) 2^-23), plus 0.01) -- the first maximum of the group with
        // the best bound gets one exact score below, the bar for everything else
#pragma unroll
        for (int i = 0; i < NC; ++i) {
            const int c = TPR * i + hh;
            const int v0 = n0 + c * 8;
            const int cnt = min(8, N - v0);
            pk[i] = *reinterpret_cast<const uint4*>(smem + G::img_off(r, c));
            float x[8];
            const uint32_t wds[4] = {pk[i].x, pk[i].y, pk[i].z, pk[i].w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x[2 * k] = __uint_as_float(wds[k] << 16);
                x[2 * k + 1] = __uint_as_float(wds[k] & 0xffff0000u);
            }
#pragma unroll
            for (int k = 0; k < 8; ++k) x[k] = k < cnt ? x[k] : -INFINITY;
            float vmax = x[0];
#pragma unroll
            for (int k = 1; k < 8; ++k) vmax = fmaxf(vmax, x[k]);
            ubc[i] = 0.f;
            vmx[i] = -INFINITY;
            hg[i] = 0u;
            if (cnt <= 0) continue;
            {
                const float mn = fmaxf(m, vmax);
                float acc_e = 0.f;
#pragma unroll
                for (int k = 0; k < 8; ++k) acc_e += fast_exp2((x[k] - mn) * kLog2eG);
                s = s * fast_exp2((m - mn) * kLog2eG) + acc_e;
                m = mn;
            }
            if constexpr (greedy) {
                if (vmax > best_s) {
                    int kk = 7;
#pragma unroll
                    for (int k = 6; k >= 0; --k) kk = (x[k] == vmax) ? k : kk;
                    best_s = vmax;
                    best_i = v0 + kk;
                    best_x = vmax;
                }
            } else {
                // bounds only (the decisions are exact scores below): every slot v of this group has
                // exact score <= x_v inv_t + c_g
                const uint32_t h = ehash(key, keyb, (uint32_t)v0 >> 3);
                const float cg = fmaf(noise_bits(h), -kBitsLn2, kNoiseC);
                ubc[i] = cg;
                vmx[i] = vmax;
                hg[i] = h;
                const float ub = vmax * inv_t + cg;
                if (ub > best_ub) {  // which group seeds the bar: its first maximum
                    int kk = 7;
#pragma unroll
                    for (int k = 6; k >= 0; --k) kk = (x[k] == vmax) ? k : kk;
                    best_ub = ub;
                    seed_g = i;
                    seed_k = kk;
                }
            }
        }
        if constexpr (!greedy) {
            GPHASE(3);
            // the tile's bar: the exact score of the first maximum of this thread's best-bound group
            // (max over the row's threads), raised to the best exact score the row's finished tiles
            // published (rowbar); both are exact scores of elements some tile reports
            // exact scores of the seed group's first maximum and of its minimum-E slot (p = h & 7:
            // E_v = E_g there, the group's largest noise); lowest index on equal scores
            float bar = -INFINITY;
            best_s = -INFINITY;
            if (seed_g >= 0) {
                uint32_t hs = 0u;
#pragma unroll
                for (int i = 0; i < NC; ++i) hs = i == seed_g ? hg[i] : hs;  // (a select chain, no scratch)
                const int c = TPR * seed_g + hh, vb = n0 + c * 8;
                const int p = (int)(hs & 7u), cnt = min(8, N - vb);
                const float eg = group_min_e(hs);
                const int ks[2] = {min(p, seed_k), max(p, seed_k)};  // ascending index
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const int k = ks[j];
                    if (k >= cnt || (j == 1 && ks[1] == ks[0])) continue;
                    const float xk = bf16_to_f32(*reinterpret_cast<const uint16_t*>(smem + G::img_off(r, c) + k * 2));
                    const float sc = noise_score(xk, inv_t, vb + k, hs, eg, key2);
                    if (sc > best_s) {
                        best_s = sc;
                        best_i = vb + k;
                        best_x = xk;
                    }
                }
                bar = best_s;
            }
#pragma unroll
            for (int o = 1; o < TPR; o <<= 1) bar = fmaxf(bar, __shfl_xor(bar, o, kWave));
            if (rowbar) bar = fmaxf(bar, bar_value(rowbar[grow]));
            // pass 2: the slots whose bound reaches the bar, as a bit mask (bit 8 i + k)
            uint32_t cm[NC / 4];
#pragma unroll
            for (int j = 0; j < NC / 4; ++j) cm[j] = 0u;
#pragma unroll
            for (int i = 0; i < NC; ++i) {
                const int v0 = n0 + (TPR * i + hh) * 8;
                const int cnt = min(8, N - v0);
                const uint32_t wds[4] = {pk[i].x, pk[i].y, pk[i].z, pk[i].w};
                // the cheap group test first (the bits bound: x inv_t + c_g, c_g's 0.01 margin covers
                // det_ln's error, the rounding is inside 1e-6 |bar|); a group that passes gets the
                // tight per-slot bound: L~ = -ln E_g by the hardware log of the exact E_g (within 1e-6
                // of -det_ln(E_g) for E_g >= 7e-9, the smallest there is) and the slack of a non-min
                // slot (E = E_g + (-det_ln U) >= E_g - 1.2e-6: exact score <= x inv_t + L + 1.4e-6 / E_g
                // + 4e-6), infinite when E_g is too small for it
                const float eps = 1e-6f * fabsf(bar);
                uint32_t bm = 0u;
                if (vmx[i] * inv_t + ubc[i] < bar - eps) continue;
                const float eg = group_min_e(hg[i]);
                const float lim = bar + hw_ln(eg) - (eg < 1e-5f ? INFINITY : 2e-4f + 5e-6f / eg) - eps;
#pragma unroll
                for (int k = 0; k < 8; ++k) {
                    const float xk = __uint_as_float((k & 1) ? (wds[k >> 1] & 0xffff0000u) : (wds[k >> 1] << 16));
                    if (k < cnt && !(xk * inv_t < lim)) bm |= 1u << k;
                }
                cm[i >> 2] |= bm << ((i & 3) * 8);
            }
            // exact scores of the candidates (minimum slots included), one per lane per trip
#pragma unroll
            for (int wd = 0; wd < NC / 4; ++wd) {
                uint32_t bm = cm[wd];
                while (bm) {
                    const int b = __builtin_ctz(bm);
                    bm &= bm - 1u;
                    const int i = wd * 4 + (b >> 3), k = b & 7;
                    const int c = TPR * i + hh;
                    const int v = n0 + c * 8 + k;
                    const float xk = bf16_to_f32(*reinterpret_cast<const uint16_t*>(smem + G::img_off(r, c) + k * 2));
                    const uint32_t h = ehash(key, keyb, (uint32_t)v >> 3);
                    const float sc = noise_score(xk, inv_t, v, h, group_min_e(h), key2);
                    if (better(sc, v, Best{best_s, best_i})) {
                        best_s = sc;
                        best_i = v;
                        best_x = xk;
                    }
                }
            }
        }
        GPHASE(4);
        // fold the row's TPR threads (adjacent lanes)
#pragma unroll
        for (int o = 1; o < TPR; o <<= 1) {
            const float os = __shfl_xor(best_s, o, kWave);
            const int oi = __shfl_xor(best_i, o, kWave);
            const float ox = __shfl_xor(best_x, o, kWave);
            if (better(os, oi, Best{best_s, best_i})) {
                best_s = os;
                best_i = oi;
                best_x = ox;
            }
            const float om = __shfl_xor(m, o, kWave), oss = __shfl_xor(s, o, kWave);
            const float mn = fmaxf(m, om);
            s = s * fast_exp2((m - mn) * kLog2eG) + oss * fast_exp2((om - mn) * kLog2eG);
            m = mn;
        }
        GPHASE(5);
        if (hh == 0) {
            if constexpr (!greedy) {
                if (rowbar && best_i != 0x7fffffff)
                    __hip_atomic_fetch_max(rowbar + grow, bar_key(best_s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            const int64_t pi = (int64_t)grow * nt + ntile;
            parts[pi] = make_float4(best_s, __int_as_float(best_i), m, s);
            part_x[pi] = best_x;
        }
    }
}

// One wave per row: fold the row's nt tile partials (ascending tile order per lane, then a
// xor tree with the (score desc, index asc) order) and finalize token + logprob.
__global__ __launch_bounds__(64) void lmhead_sample_merge_kernel(const float4* __restrict__ parts,
                                                                 const float* __restrict__ part_x, int nt,
                                                                 int32_t* __restrict__ tokens,
                                                                 float* __restrict__ logp_out,
                                                                 unsigned* __restrict__ rowbar) {
    const int row = blockIdx.x, lane = threadIdx.x;
    if (rowbar && lane == 0) rowbar[row] = 0u;  // re-arm the row's cross-tile bar (every tile is done)
    Best b{-INFINITY, 0x7fffffff};
    float bx = __builtin_nanf(""), m = -1e30f, s = 0.f;
    // 8 partials per lane in flight before folding them (the fold is a dependent chain)
    for (int j0 = lane; j0 < nt; j0 += 8 * 64) {
        float4 pv[8];
        float px[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int j = j0 + u * 64;
            pv[u] = j < nt ? parts[(int64_t)row * nt + j] : make_float4(-INFINITY, __int_as_float(0x7fffffff), -1e30f, 0.f);
            px[u] = j < nt ? part_x[(int64_t)row * nt + j] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const float4 p = pv[u];
            const int idx = __float_as_int(p.y);
            if (better(p.x, idx, b)) {
                b = Best{p.x, idx};
                bx = px[u];
            }
            const float mn = fmaxf(m, p.z);
            s = s * fast_exp2((m - mn) * kLog2eG) + p.w * fast_exp2((p.z - mn) * kLog2eG);
            m = mn;
        }
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float os = __shfl_xor(b.score, off, kWave);
        const int oi = __shfl_xor(b.idx, off, kWave);
        const float ox = __shfl_xor(bx, off, kWave);
        if (better(os, oi, b)) {
            b = Best{os, oi};
            bx = ox;
        }
        const float om = __shfl_xor(m, off, kWave), oss = __shfl_xor(s, off, kWave);
        const float mn = fmaxf(m, om);
        s = s * fast_exp2((m - mn) * kLog2eG) + oss * fast_exp2((om - mn) * kLog2eG);
        m = mn;
    }
    if (lane == 0) {
        tokens[row] = b.idx;
        if (logp_out) logp_out[row] = bx - (m + fast_log2(s) * kLn2G);
    }
}

// LDS store / load of 16 B by inline asm: the compiler puts s_waitcnt vmcnt(0) in front of any LDS
// access it can see while an LDS-DMA copy may be in flight, which would drain the next steps'
// copies at the epilogue; these the caller orders itself (lgkmcnt waits + barriers)
__device__ __forceinline__ void lds_st16(float4* p, f32x4 v) {
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)(char*)p;
    asm volatile("ds_write_b128 %0, %1" ::"v"(a), "v"(v) : "memory");
}
__device__ __forceinline__ f32x4 lds_ld16(const float4* p) {
    const uint32_t a = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const char*)(const char*)p;
    f32x4 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(a) : "memory");
    return v;
}

// ---- learner forward, persistent form (the default of skyrl_lmhead_logprob_fwd) ---------------
// One 512-thread workgroup per CU walks the tiles q = i nwg + wg of the grouped order (wg in the
// XCD-contiguous numbering, so in every round an XCD's 32 workgroups hold 8 M tiles x 4 N tiles of
// one group) with ONE K pipeline across its tiles: global step g = i nk + t stages H in LDS stage
// g & 1 and W in stage g % 3 (pipe 12's staging: H(g + 1) and W(g + 2) in flight while step g
// computes), so the next tile's first copies are in flight through this tile's last steps and its
// epilogue instead of after it.
// The MFMAs take the operands swapped (A = the W fragment, B = the H fragment), so lane l of wave
// (wm, wn) holds, for each of its 8 tokens m0 + 128 wm + 16 tb + (l & 15), the 16 columns
// n0 + 64 wn + 16 vb + 4 (l >> 4) + r (vb, r < 4). The epilogue runs from registers (no LDS image):
// the bf16 logits of a token's 16 columns fold into one (m, S, W) state per lane, two xor merges
// join the lane groups, and the four column waves' states meet in the H stage the last step read (a
// 16 KB scratch until step g + 1 restages it), merged in wn order by one thread per token into the
// tile's state. The label logit is not taken here: lmhead_label_merge_kernel recomputes it with the
// same MFMA chain, bit for bit.
// CP (skyrl_variant lmhead_persist - 1): where a wave issues its 8 copies of a step: 0 all right
// after the step's barrier; 1 the second wave of each SIMD (waves 4-7) after its first four MFMA
// groups; 2 one copy per MFMA group; 3 role split: waves 0-3 copy all of H(g + 1) after the
// barrier, waves 4-7 all of W(g + 2) after their first four MFMA groups.
// EPI: EPI_LOGPROB (the learner forward: per (tile, token) the softmax state (m, S, W) after the
// reference's bf16 division by T, into parts[ntile][M]) or EPI_GREEDY (the decode side's greedy
// step: per (token, tile) the first maximum and the raw (max, sum-exp), into parts[M][nt] and
// part_x, lmhead_sample_merge_kernel's partials).
template <int EPI, bool HAS_T, int CP>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) void lmhead_logprob_pkernel(
    const uint16_t* __restrict__ H, int64_t ldh, const uint16_t* __restrict__ W, int64_t ldw, int M, int N, int K,
    int mt, int nt, int gm, float temp, float4* __restrict__ parts, float* __restrict__ part_x) {
    constexpr int NST = EPI == EPI_GREEDY ? 2 : 1;  // stores of a storing wave's epilogue
    using G = Geo<256, 64, 2>;
    constexpr int kT = 32768, kWBase = 2 * kT, kRow = 128;
    __shared__ __attribute__((aligned(16))) char smem[163840];
    const int nwg = gridDim.x, orig = blockIdx.x, xcd = orig & 7, q = nwg >> 3, rr = nwg & 7;
    const int wg = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (orig >> 3);
    const int ntiles = mt * nt;
    const int my = wg < ntiles ? (ntiles - 1 - wg) / nwg + 1 : 0;
    if (my == 0) return;
    const int nk = K / 64;  // >= 2 (host)
    const int nsteps = my * nk;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int wm = w & 1, wn = w >> 1;
    auto tile_mn = [&](int i, int& mtile, int& ntile) {
        const int qq = min(i, my - 1) * nwg + wg;
        if (gm <= 0 || gm >= mt) {
            mtile = qq % mt;
            ntile = qq / mt;
        } else {
            const int per = gm * nt, gi = qq / per, r = qq - gi * per, gsz = min(gm, mt - gi * gm);
            mtile = gi * gm + r % gsz;
            ntile = r / gsz;
        }
    };
    // Staging: a step's copies are 16 pieces of 8 rows x 128 B per operand (lane -> row lane >> 3,
    // 16-B chunk lane & 7 holding logical chunk (lane & 7) ^ swz(row)). CP 0-2: wave w copies H
    // rows and W rows 32 w .. 32 w + 31 (4 pieces each); CP 3 (role split): waves 0-3 copy H only
    // and waves 4-7 W only, rows 64 (w & 3) .. + 63 (8 pieces). Offsets are 32-bit element offsets
    // of the current (oc) and the next (ox) tile (the host takes this path only when M ldh,
    // N ldw < 2^31); CP 0-2 keep H in [0, 4) and W in [4, 8).
    constexpr bool SPLIT = CP == 3;
    const bool hrole = !SPLIT || __builtin_amdgcn_readfirstlane(w) < 4;  // SPLIT: this wave copies H
    int srow[8], scol[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        srow[j] = SPLIT ? (w & 3) * 64 + j * 8 + (lane >> 3) : (w * 4 + (j & 3)) * 8 + (lane >> 3);
        scol[j] = ((lane & 7) ^ G::swz(srow[j])) * 8;
    }
    uint32_t oc[8], ox[8];
    auto offs = [&](int i, uint32_t (&o)[8]) {
        int mtile, ntile;
        tile_mn(i, mtile, ntile);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const bool isw = SPLIT ? !hrole : j >= 4;
            o[j] = isw ? (uint32_t)min(ntile * 256 + srow[j], N - 1) * (uint32_t)ldw + (uint32_t)scol[j]
                       : (uint32_t)min(mtile * BM + srow[j], M - 1) * (uint32_t)ldh + (uint32_t)scol[j];
        }
    };
    // LDS byte offset of this wave's piece j inside a stage
    auto pdst = [&](int j) { return SPLIT ? ((w & 3) * 8 + j) * 1024 : (w * 4 + (j & 3)) * 1024; };
    // piece j: an H piece of step g + 1 or a W piece of step g + 2 (when those steps exist)
    auto copy_piece = [&](auto j_tag, int g, int t, int hs, int ws) __attribute__((always_inline)) {
        constexpr int j = decltype(j_tag)::value;
        const bool isw = SPLIT ? !hrole : j >= 4;
        if (!isw) {
            if (g + 1 >= nsteps) return;
            const bool cur = t + 1 < nk;
            __builtin_amdgcn_global_load_lds((gbl_void*)(H + (cur ? oc[j] : ox[j]) + (cur ? t + 1 : 0) * 64),
                                             (lds_void*)(smem + (hs ^ 1) * kT + pdst(j)), 16, 0, 0);
        } else {
            if (g + 2 >= nsteps) return;
            const bool cur = t + 2 < nk;
            const int w2 = ws == 0 ? 2 : ws - 1;  // (g + 2) % 3
            __builtin_amdgcn_global_load_lds((gbl_void*)(W + (cur ? oc[j] : ox[j]) + (cur ? t + 2 : t + 2 - nk) * 64),
                                             (lds_void*)(smem + kWBase + w2 * kT + pdst(j)), 16, 0, 0);
        }
    };
    // the prologue's copies: phase 0 H(0) and W(0), phase 1 W(1) (every W(1) piece after every
    // W(0) piece, so the top of step 0 may leave exactly the W(1) pieces outstanding)
    auto copy0 = [&](auto j_tag, int phase) __attribute__((always_inline)) {
        constexpr int j = decltype(j_tag)::value;
        const bool isw = SPLIT ? !hrole : j >= 4;
        if (!isw) {
            if (phase == 0) __builtin_amdgcn_global_load_lds((gbl_void*)(H + oc[j]), (lds_void*)(smem + pdst(j)), 16, 0, 0);
        } else if (phase == 0) {
            __builtin_amdgcn_global_load_lds((gbl_void*)(W + oc[j]), (lds_void*)(smem + kWBase + pdst(j)), 16, 0, 0);
        } else if (nsteps > 1) {
            __builtin_amdgcn_global_load_lds((gbl_void*)(W + oc[j] + 64), (lds_void*)(smem + kWBase + kT + pdst(j)), 16, 0, 0);
        }
    };
    auto copy_all = [&](int g, int t, int hs, int ws) __attribute__((always_inline)) {
        copy_piece(std::integral_constant<int, 0>{}, g, t, hs, ws);
        copy_piece(std::integral_constant<int, 1>{}, g, t, hs, ws);
        copy_piece(std::integral_constant<int, 2>{}, g, t, hs, ws);
        copy_piece(std::integral_constant<int, 3>{}, g, t, hs, ws);
        copy_piece(std::integral_constant<int, 4>{}, g, t, hs, ws);
        copy_piece(std::integral_constant<int, 5>{}, g, t, hs, ws);
        copy_piece(std::integral_constant<int, 6>{}, g, t, hs, ws);
        copy_piece(std::integral_constant<int, 7>{}, g, t, hs, ws);
    };
    // CP 1: the second wave of each SIMD copies mid-step; CP 3: the W waves do
    const bool late = (CP == 1 && __builtin_amdgcn_readfirstlane(w) >= 4) || (SPLIT && !hrole);
    int aoff[2], boff[2];
    {
        const int sw = G::swz(lane & 15);
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = (ks * 4 + (lane >> 4)) ^ sw;
            aoff[ks] = (wm * 128 + (lane & 15)) * kRow + c * 16;
            boff[ks] = kWBase + (wn * 64 + (lane & 15)) * kRow + c * 16;
        }
    }
    f32x4 acc[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    offs(0, oc);
    offs(1, ox);
    int mtile, ntile;
    tile_mn(0, mtile, ntile);
#pragma unroll
    for (int phase = 0; phase < 2; ++phase) {
        copy0(std::integral_constant<int, 0>{}, phase);
        copy0(std::integral_constant<int, 1>{}, phase);
        copy0(std::integral_constant<int, 2>{}, phase);
        copy0(std::integral_constant<int, 3>{}, phase);
        copy0(std::integral_constant<int, 4>{}, phase);
        copy0(std::integral_constant<int, 5>{}, phase);
        copy0(std::integral_constant<int, 6>{}, phase);
        copy0(std::integral_constant<int, 7>{}, phase);
    }
    int i = 0, t = 0, hs = 0, ws = 0;
    bool stored = false;  // this wave issued the previous step's state store (one more vmcnt entry)
    for (int g = 0; g < nsteps; ++g) {
        // H(g) and W(g) have landed once only the younger W(g + 1) copies (if issued) and the
        // previous epilogue's store (1) may be outstanding: 4 W pieces per wave (CP 0-2), 8 for a
        // W wave and none for an H wave (CP 3, whose H(g) was issued after W(g + 1))
        if (g + 1 < nsteps && !(SPLIT && hrole)) {
            if constexpr (SPLIT) {
                wait_vmcnt<8>();  // W waves never store
            } else {
                if (stored) wait_vmcnt<4 + NST>();
                else wait_vmcnt<4>();
            }
        } else {
            if (stored) wait_vmcnt<NST>();
            else wait_vmcnt<0>();
        }
        stored = false;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const char* sa = smem + hs * kT;
        const char* sbw = smem + ws * kT;  // + boff's kWBase
        // H(g + 1) and W(g + 2): this tile's next steps or the next tile's first ones
        if (CP == 0 || ((CP == 1 || CP == 3) && !late)) copy_all(g, t, hs, ws);
        // pipe 12's fragment pipeline (groups of 2 H x 4 W fragments), operands swapped
        bf16x8 bq[2][4], aq[2][2];
        auto ldA = [&](int ks, int mp, bf16x8 (&dst)[2]) {
#pragma unroll
            for (int u = 0; u < 2; ++u)
                dst[u] = *reinterpret_cast<const bf16x8*>(sa + aoff[ks] + (2 * mp + u) * 16 * kRow);
        };
        auto ldB = [&](int ks) {
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) bq[ks][nb] = *reinterpret_cast<const bf16x8*>(sbw + boff[ks] + nb * 16 * kRow);
        };
        ldB(0);
        ldA(0, 0, aq[0]);
#pragma unroll
        for (int gg = 0; gg < 8; ++gg) {
            const int ks = gg / 4, mp = gg % 4;
            if constexpr (CP == 2) {
                switch (gg) {
                    case 0: copy_piece(std::integral_constant<int, 0>{}, g, t, hs, ws); break;
                    case 1: copy_piece(std::integral_constant<int, 1>{}, g, t, hs, ws); break;
                    case 2: copy_piece(std::integral_constant<int, 2>{}, g, t, hs, ws); break;
                    case 3: copy_piece(std::integral_constant<int, 3>{}, g, t, hs, ws); break;
                    case 4: copy_piece(std::integral_constant<int, 4>{}, g, t, hs, ws); break;
                    case 5: copy_piece(std::integral_constant<int, 5>{}, g, t, hs, ws); break;
                    case 6: copy_piece(std::integral_constant<int, 6>{}, g, t, hs, ws); break;
                    default: copy_piece(std::integral_constant<int, 7>{}, g, t, hs, ws); break;
                }
            }
            if ((CP == 1 || CP == 3) && late && gg == 4) copy_all(g, t, hs, ws);
            if (gg + 1 < 8) {
                if ((gg + 1) % 4 == 0) ldB((gg + 1) / 4);
                ldA((gg + 1) / 4, (gg + 1) % 4, aq[(gg + 1) & 1]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int nb = 0; nb < 4; ++nb)
                    acc[2 * mp + u][nb] =
                        __builtin_amdgcn_mfma_f32_16x16x32_bf16(bq[ks][nb], aq[gg & 1][u], acc[2 * mp + u][nb], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (t + 1 == nk) {
            // ---- epilogue of tile i: every wave's reads of H stage hs are done, it is the scratch
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            float4* scr = reinterpret_cast<float4*>(smem + hs * kT);  // [256 tokens][4 column waves]
            const int n0 = ntile * 256, m0 = mtile * BM;
            const int cbase = n0 + wn * 64 + (lane >> 4) * 4;
            if constexpr (EPI == EPI_LOGPROB || EPI == EPI_LOGPROB_NOENT) {
                // a token's state over this wave's 64 columns: the max over the four lane groups
                // first, then every exponential against it (no rescaling merges); sums joined by two
                // xor adds. FULL: every column inside V (no masks, no clamps).
                auto token_states = [&](auto full_tag) __attribute__((always_inline)) {
                    constexpr bool FULL = decltype(full_tag)::value;
    #pragma unroll
                    for (int tb = 0; tb < 8; ++tb) {
                        float x[16];
    #pragma unroll
                        for (int vb = 0; vb < 4; ++vb)
    #pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                float v = bf16_to_f32(f32_to_bf16(acc[tb][vb][r]));  // the logits the reference writes
                                if constexpr (HAS_T) v = Elem<uint16_t>::apply_t(v, temp, true);
                                if constexpr (!FULL) v = cbase + vb * 16 + r < N ? v : -INFINITY;
                                x[vb * 4 + r] = v;
                            }
                        float mx = fmaxf(fmaxf(x[0], x[1]), x[2]);
    #pragma unroll
                        for (int k = 3; k < 15; k += 2) mx = fmaxf(fmaxf(mx, x[k]), x[k + 1]);
                        mx = fmaxf(mx, x[15]);
                        mx = fmaxf(mx, __shfl_xor(mx, 16, kWave));
                        mx = fmaxf(mx, __shfl_xor(mx, 32, kWave));
                        if constexpr (!FULL) mx = fmaxf(mx, -3.402823466e38f);  // columns all outside V: finite
                        const float c = -mx * kLog2e;
                        float sa = 0.f, sb = 0.f, wa = 0.f, wb = 0.f;  // two chains each
    #pragma unroll
                        for (int k = 0; k < 16; ++k) {
                            float y = fmaf(x[k], kLog2e, c);
                            if constexpr (!FULL) y = fmaxf(y, kDLow);
                            const float e = fast_exp2(y);
                            if (k & 1) {
                                sb += e;
                                if constexpr (EPI == EPI_LOGPROB) wb = fmaf(e, y, wb);
                            } else {
                                sa += e;
                                if constexpr (EPI == EPI_LOGPROB) wa = fmaf(e, y, wa);
                            }
                        }
                        float ss = sa + sb, ww = wa + wb;  // W only for the entropy (EPI_LOGPROB)
                        ss += __shfl_xor(ss, 16, kWave);
                        ss += __shfl_xor(ss, 32, kWave);
                        if constexpr (EPI == EPI_LOGPROB) {
                            ww += __shfl_xor(ww, 16, kWave);
                            ww += __shfl_xor(ww, 32, kWave);
                        }
                        if (lane < 16) lds_st16(scr + (wm * 128 + tb * 16 + lane) * 4 + wn, f32x4{mx, ss, ww, 0.f});
                    }
                };
                if (n0 + 256 <= N) token_states(std::true_type{});
                else token_states(std::false_type{});
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (w < 4) {
                    const int tok = threadIdx.x;  // 0 .. 255
                    const f32x4 s0 = lds_ld16(scr + tok * 4 + 0), s1 = lds_ld16(scr + tok * 4 + 1);
                    const f32x4 s2 = lds_ld16(scr + tok * 4 + 2), s3 = lds_ld16(scr + tok * 4 + 3);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                    SoftState st{s0[0], s0[1], s0[2]};
                    state_merge(st, SoftState{s1[0], s1[1], s1[2]});
                    state_merge(st, SoftState{s2[0], s2[1], s2[2]});
                    state_merge(st, SoftState{s3[0], s3[1], s3[2]});
                    // one store instruction per wave whenever any of its tokens is inside M
                    stored = m0 + w * 64 < M;
                    if (m0 + tok < M) parts[(int64_t)ntile * M + m0 + tok] = make_float4(st.m, st.s, st.w, __builtin_nanf(""));
                }
            } else {
                // greedy: the first maximum of the token's 64 columns (lane order is column order,
                // then the lower index on equal values across lane groups) and the raw sum-exp
                // against it
                auto token_argmax = [&](auto full_tag) __attribute__((always_inline)) {
                    constexpr bool FULL = decltype(full_tag)::value;
#pragma unroll
                    for (int tb = 0; tb < 8; ++tb) {
                        float x[16];
#pragma unroll
                        for (int vb = 0; vb < 4; ++vb)
#pragma unroll
                            for (int r = 0; r < 4; ++r) {
                                float v = bf16_to_f32(f32_to_bf16(acc[tb][vb][r]));
                                if constexpr (!FULL) v = cbase + vb * 16 + r < N ? v : -INFINITY;
                                x[vb * 4 + r] = v;
                            }
                        float bx = x[0];
                        int bk = 0;
#pragma unroll
                        for (int k = 1; k < 16; ++k) {
                            if (x[k] > bx) {
                                bx = x[k];
                                bk = k;
                            }
                        }
                        int bi = cbase + (bk >> 2) * 16 + (bk & 3);
#pragma unroll
                        for (int off = 16; off < 64; off <<= 1) {
                            const float ox = __shfl_xor(bx, off, kWave);
                            const int oi = __shfl_xor(bi, off, kWave);
                            if (ox > bx || (ox == bx && oi < bi)) {
                                bx = ox;
                                bi = oi;
                            }
                        }
                        // columns all outside V: a finite floor whose -mx log2e does not overflow
                        // (-inf x then gives exp2(-inf) = 0, never inf - inf)
                        const float mx = FULL ? bx : fmaxf(bx, -1e30f);
                        const float c = -mx * kLog2e;
                        float sa = 0.f, sb = 0.f;
#pragma unroll
                        for (int k = 0; k < 16; k += 2) {
                            sa += fast_exp2(fmaf(x[k], kLog2e, c));
                            sb += fast_exp2(fmaf(x[k + 1], kLog2e, c));
                        }
                        float ss = sa + sb;
                        ss += __shfl_xor(ss, 16, kWave);
                        ss += __shfl_xor(ss, 32, kWave);
                        if (lane < 16)
                            lds_st16(scr + (wm * 128 + tb * 16 + lane) * 4 + wn, f32x4{bx, __int_as_float(bi), mx, ss});
                    }
                };
                if (n0 + 256 <= N) token_argmax(std::true_type{});
                else token_argmax(std::false_type{});
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                __builtin_amdgcn_s_barrier();
                if (w < 4) {
                    const int tok = threadIdx.x;  // 0 .. 255
                    f32x4 r[4];
#pragma unroll
                    for (int j = 0; j < 4; ++j) r[j] = lds_ld16(scr + tok * 4 + j);
                    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                    __builtin_amdgcn_sched_barrier(0);
                    float bx = r[0][0], m = r[0][2], sm = r[0][3];
                    int bi = __float_as_int(r[0][1]);
#pragma unroll
                    for (int j = 1; j < 4; ++j) {
                        if (r[j][0] > bx) {  // column waves in column order: strict '>' keeps the first
                            bx = r[j][0];
                            bi = __float_as_int(r[j][1]);
                        }
                        const float mn = fmaxf(m, r[j][2]);
                        sm = sm * fast_exp2((m - mn) * kLog2e) + r[j][3] * fast_exp2((r[j][2] - mn) * kLog2e);
                        m = mn;
                    }
                    stored = m0 + w * 64 < M;
                    if (m0 + tok < M) {
                        const int64_t pi = (int64_t)(m0 + tok) * nt + ntile;
                        parts[pi] = make_float4(bx, __int_as_float(bi), m, sm);
                        part_x[pi] = bx;
                    }
                }
            }
            // the next tile
#pragma unroll
            for (int a = 0; a < 8; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
            ++i;
            t = 0;
#pragma unroll
            for (int j = 0; j < 8; ++j) oc[j] = ox[j];
            offs(i + 1, ox);
            tile_mn(i, mtile, ntile);
        } else {
            ++t;
        }
        hs ^= 1;
        ws = ws == 2 ? 0 : ws + 1;
    }
}

// The learner forward's finish, one wave per 16 tokens. The label logit by the tile kernel's own
// MFMA chain: A = the 16 label rows of W, B = the 16 token rows of H, the k chunks of 32 in the
// same order from a zero accumulator, so D[i][i] is the tile kernel's accumulator for (token i,
// label i) bit for bit; rounded to bf16 and divided by T as there (NaN for a label outside [0, V),
// as logprob.hip). Then the token's nt tile states: lane group q merges the tiles
// [q nt / 4, (q + 1) nt / 4) in order, two xor merges join the groups, finalize.
__global__ __launch_bounds__(64) void lmhead_label_merge_kernel(
    const uint16_t* __restrict__ H, int64_t ldh, const uint16_t* __restrict__ W, int64_t ldw, int T, int V, int K,
    const int64_t* __restrict__ labels, int64_t lstride, float temp, int has_t, const float4* __restrict__ parts, int nt,
    float* __restrict__ logp_out, float* __restrict__ ent_out, float* __restrict__ lse_out) {
    const int lane = threadIdx.x, i = lane & 15, grp = lane >> 4;
    const int tok = min((int)blockIdx.x * 16 + i, T - 1);
    const int64_t lab = labels[(int64_t)tok * lstride];
    const bool valid = lab >= 0 && lab < V;
    const uint16_t* wr = W + (valid ? lab : 0) * ldw + grp * 8;
    const uint16_t* hr = H + (int64_t)tok * ldh + grp * 8;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nkc = K / 32;
    int kc = 0;
    for (; kc + 4 <= nkc; kc += 4) {
        bf16x8 a[4], b[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            a[u] = *reinterpret_cast<const bf16x8*>(wr + (kc + u) * 32);
            b[u] = *reinterpret_cast<const bf16x8*>(hr + (kc + u) * 32);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[u], acc, 0, 0, 0);
    }
    for (; kc < nkc; ++kc)
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<const bf16x8*>(wr + kc * 32),
                                                      *reinterpret_cast<const bf16x8*>(hr + kc * 32), acc, 0, 0, 0);
    // lane L holds D rows 4 (L >> 4) + r: row i's diagonal element is lane ((i >> 2) << 4) | i's r = i & 3
    const int r3 = lane & 3;
    const float dsel = r3 == 0 ? acc[0] : r3 == 1 ? acc[1] : r3 == 2 ? acc[2] : acc[3];
    const float d = __shfl(dsel, ((i >> 2) << 4) | i, kWave);
    float xl = bf16_to_f32(f32_to_bf16(d));
    if (has_t) xl = Elem<uint16_t>::apply_t(xl, temp, true);
    if (!valid) xl = __builtin_nanf("");
    SoftState st;
    state_init(st);
    const int j1 = (grp + 1) * nt / 4;
    int j = grp * nt / 4;
    for (; j + 8 <= j1; j += 8) {
        float4 c[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) c[u] = parts[(int64_t)(j + u) * T + tok];
#pragma unroll
        for (int u = 0; u < 8; ++u) state_merge(st, SoftState{c[u].x, c[u].y, c[u].z});
    }
    for (; j < j1; ++j) {
        const float4 c = parts[(int64_t)j * T + tok];
        state_merge(st, SoftState{c.x, c.y, c.z});
    }
#pragma unroll
    for (int off = 16; off < 64; off <<= 1) {
        SoftState o;
        o.m = __shfl_xor(st.m, off, kWave);
        o.s = __shfl_xor(st.s, off, kWave);
        o.w = __shfl_xor(st.w, off, kWave);
        state_merge(st, o);
    }
    if (lane < 16 && (int)blockIdx.x * 16 + lane < T) finalize_row(st, xl, tok, logp_out, ent_out, lse_out);
}

inline int tiles(int n, int b) { return (n + b - 1) / b; }

using GemmKernel = void (*)(const uint16_t*, int64_t, const uint16_t*, int64_t, int, int, int, int, uint16_t*, int64_t,
                            float, uint64_t, const int64_t*, int64_t, float4*, float*, int, const int64_t*, int64_t,
                            unsigned*);
int group_for(int mt) { return knobs().lmhead_group > 0 && knobs().lmhead_group < mt ? knobs().lmhead_group : 0; }
int tile_threads(int pipe) { return pipe == 13 ? 256 : 2 * (pipe == 1 ? 128 : 256); }
// the pipeline for these operands: pipe 13 addresses them with 32-bit element offsets
int pipe_for(int64_t M, int64_t ldh, int64_t N, int64_t ldw) {
    if (knobs().lmhead_pipe == 13 && (M * ldh >= (int64_t(1) << 31) || N * ldw >= (int64_t(1) << 31))) return 12;
    return knobs().lmhead_pipe;
}
int tile_n(int pipe) { return pipe == 1 ? 128 : 256; }  // pipe 3: 256, staggered copies
template <int EPI>
GemmKernel pick_kernel(int pipe) {
    switch (pipe) {
        case 1: return lmhead_gemm_kernel<EPI, 128, 32, 3, 0, 0>;
        case 2: return lmhead_gemm_kernel<EPI, 256, 32, 4, 0, 0>;
        case 3: return lmhead_gemm_kernel<EPI, 256, 64, 2, 1, 0>;
        case 4: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 1>;
        case 5: return lmhead_gemm_kernel<EPI, 256, 64, 2, 1, 1>;
        case 6: return lmhead_gemm_kernel<EPI, 256, 32, 4, 0, 1>;
        case 7: return lmhead_gemm_kernel<EPI, 256, 32, 3, 0, 1>;
        case 8: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 2>;
        case 9: return lmhead_gemm_kernel<EPI, 256, 32, 4, 0, 2>;
        case 10: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 3>;
        case 11: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 4>;
        case 12: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 5>;
        case 13: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 6>;
        case 14: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 7>;
        default: return lmhead_gemm_kernel<EPI, 256, 64, 2, 0, 0>;
    }
}

int check_operands(const void* h, int64_t ldh, const void* w, int64_t ldw, int M, int N, int K) {
    SKYRL_REQUIRE(M >= 0 && N > 0 && K > 0, "lmhead_gemm: bad sizes");
    SKYRL_REQUIRE(K % 64 == 0, "lmhead_gemm: K must be a multiple of 64");
    SKYRL_REQUIRE(ldh >= K && ldw >= K && ldh % 8 == 0 && ldw % 8 == 0, "lmhead_gemm: row strides must be >= K and 16-B multiples");
    SKYRL_REQUIRE(h && w, "lmhead_gemm: null operand");
    SKYRL_REQUIRE((reinterpret_cast<uintptr_t>(h) & 15) == 0 && (reinterpret_cast<uintptr_t>(w) & 15) == 0,
                  "lmhead_gemm: operands must be 16-B aligned");
    return SKYRL_OK;
}

}  // namespace

}  // namespace skyrl

using namespace skyrl;

extern "C" int skyrl_lmhead_gemm(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight, int32_t M,
                                 int32_t N, int32_t K, void* out, int64_t ld_out, void* stream) {
    int rc = check_operands(hidden, ld_hidden, weight, ld_weight, M, N, K);
    if (rc) return rc;
    if (M == 0) return SKYRL_OK;
    SKYRL_REQUIRE(out && ld_out >= N, "lmhead_gemm: bad output");
    const int pipe = pipe_for(M, ld_hidden, N, ld_weight);
    const int bn = tile_n(pipe), mt = tiles(M, BM), nt = tiles(N, bn);
    hipLaunchKernelGGL(pick_kernel<EPI_STORE>(pipe), dim3(mt * nt), dim3(tile_threads(pipe)), 0, as_stream(stream),
                       reinterpret_cast<const uint16_t*>(hidden), ld_hidden, reinterpret_cast<const uint16_t*>(weight),
                       ld_weight, M, N, K, mt | (group_for(mt) << 16), reinterpret_cast<uint16_t*>(out), ld_out, 1.f, 0ull, nullptr, 0ll,
                       nullptr, nullptr, nt, nullptr, 0ll, nullptr);
    return check_launch("lmhead_gemm_kernel<store>");
}

// Sampling workspace: the cross-tile row bars first, in a fixed region (the same place for every
// row count: zero at allocation, re-armed by the merge kernel; calls of more rows than the region
// holds run without them), then the tile partials.
constexpr int kBarRows = 16384;
constexpr size_t kBarBytes = (size_t)kBarRows * 4;

extern "C" size_t skyrl_lmhead_sample_workspace_bytes(int32_t M, int32_t V) {
    const size_t n = (size_t)(M > 0 ? M : 1) * tiles(V > 0 ? V : 1, 128);  // the smallest tile width
    return kBarBytes + n * sizeof(float4) + n * sizeof(float) + 256;
}

extern "C" int skyrl_lmhead_sample(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight,
                                   int32_t M, int32_t V, int32_t K, float temperature, uint64_t seed,
                                   const int64_t* seq_ids, int64_t step, int32_t* tokens_out, float* logp_out,
                                   void* workspace, void* stream) {
    int rc = check_operands(hidden, ld_hidden, weight, ld_weight, M, V, K);
    if (rc) return rc;
    if (M == 0) return SKYRL_OK;
    SKYRL_REQUIRE(tokens_out && workspace, "lmhead_sample: null pointer");
    SKYRL_REQUIRE(temperature >= 0.f, "lmhead_sample: temperature must be >= 0");
    SKYRL_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "lmhead_sample: workspace must be 16-B aligned");
    const int pipe = pipe_for(M, ld_hidden, V, ld_weight);
    const int bn = tile_n(pipe), mt = tiles(M, BM), nt = tiles(V, bn);
    unsigned* rowbar = M <= kBarRows ? reinterpret_cast<unsigned*>(workspace) : nullptr;
    float4* parts = reinterpret_cast<float4*>(reinterpret_cast<char*>(workspace) + kBarBytes);
    float* part_x = reinterpret_cast<float*>(parts + (size_t)M * nt);
    const bool greedy = temperature == 0.f;
    const float inv_t = greedy ? 1.f : 1.0f / temperature;
    if (greedy) rowbar = nullptr;
    if (greedy && knobs().lmhead_persist != 0 && K >= 128 && (int64_t)M * ld_hidden < (int64_t(1) << 31) &&
        (int64_t)V * ld_weight < (int64_t(1) << 31)) {
        // the persistent tile kernel when it has at least four rounds of tiles (decode batches of
        // 512+ rows); below that one tile per workgroup balances better
        const int pmt = tiles(M, BM), pnt = tiles(V, 256);
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return fail(SKYRL_ERR_LAUNCH, "lmhead_sample: device query failed");
        if (pmt * pnt >= 4 * ncu) {
            const int cp = knobs().lmhead_persist - 1;
            auto pk = cp == 0   ? lmhead_logprob_pkernel<EPI_GREEDY, false, 0>
                      : cp == 1 ? lmhead_logprob_pkernel<EPI_GREEDY, false, 1>
                      : cp == 2 ? lmhead_logprob_pkernel<EPI_GREEDY, false, 2>
                                : lmhead_logprob_pkernel<EPI_GREEDY, false, 3>;
            float* px = reinterpret_cast<float*>(parts + (size_t)M * pnt);
            hipLaunchKernelGGL(pk, dim3(min(pmt * pnt, ncu)), dim3(512), 0, as_stream(stream),
                               reinterpret_cast<const uint16_t*>(hidden), ld_hidden, reinterpret_cast<const uint16_t*>(weight),
                               ld_weight, M, V, K, pmt, pnt, group_for(pmt), 1.f, parts, px);
            rc = check_launch("lmhead_logprob_pkernel<greedy>");
            if (rc) return rc;
            hipLaunchKernelGGL(lmhead_sample_merge_kernel, dim3(M), dim3(64), 0, as_stream(stream), parts, px, pnt,
                               tokens_out, logp_out, nullptr);
            return check_launch("lmhead_sample_merge_kernel");
        }
    }
    auto kern = greedy ? pick_kernel<EPI_GREEDY>(pipe) : pick_kernel<EPI_SAMPLE>(pipe);
    hipLaunchKernelGGL(kern, dim3(mt * nt), dim3(tile_threads(pipe)), 0, as_stream(stream), reinterpret_cast<const uint16_t*>(hidden),
                       ld_hidden, reinterpret_cast<const uint16_t*>(weight), ld_weight, M, V, K, mt | (group_for(mt) << 16), nullptr, 0ll, inv_t,
                       seed, seq_ids, step, parts, part_x, nt, nullptr, 0ll, rowbar);
    rc = check_launch("lmhead_gemm_kernel<sample>");
    if (rc) return rc;
    hipLaunchKernelGGL(lmhead_sample_merge_kernel, dim3(M), dim3(64), 0, as_stream(stream), parts, part_x, nt, tokens_out,
                       logp_out, rowbar);
    return check_launch("lmhead_sample_merge_kernel");
}

extern "C" size_t skyrl_lmhead_logprob_workspace_bytes(int32_t T, int32_t V) {
    return (size_t)(T > 0 ? T : 1) * tiles(V > 0 ? V : 1, 128) * sizeof(float4) + 256;
}

extern "C" int skyrl_lmhead_logprob_fwd(const void* hidden, int64_t ld_hidden, const void* weight, int64_t ld_weight,
                                        int32_t T, int32_t V, int32_t K, const int64_t* labels, int64_t label_stride,
                                        float temperature, float* logp_out, float* entropy_out, float* lse_out,
                                        void* workspace, void* stream) {
    int rc = check_operands(hidden, ld_hidden, weight, ld_weight, T, V, K);
    if (rc) return rc;
    if (T == 0) return SKYRL_OK;
    SKYRL_REQUIRE(labels && logp_out && workspace, "lmhead_logprob_fwd: null pointer");
    SKYRL_REQUIRE(temperature > 0.f, "lmhead_logprob_fwd: temperature must be > 0");
    SKYRL_REQUIRE((reinterpret_cast<uintptr_t>(workspace) & 15) == 0, "lmhead_logprob_fwd: workspace must be 16-B aligned");
    float4* states = reinterpret_cast<float4*>(workspace);
    if (knobs().lmhead_persist != 0 && K >= 128 && (int64_t)T * ld_hidden < (int64_t(1) << 31) &&
        (int64_t)V * ld_weight < (int64_t(1) << 31)) {
        // the persistent tile kernel (one workgroup per CU) + the label / merge launch
        const int mt = tiles(T, BM), nt = tiles(V, 256);
        int dev = 0, ncu = 256;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            return fail(SKYRL_ERR_LAUNCH, "lmhead_logprob_fwd: device query failed");
        const int grid = min(mt * nt, ncu);
        const int cp = knobs().lmhead_persist - 1;
        const bool ht = temperature != 1.0f;
        auto pk = !entropy_out && cp == 3 ? (ht ? lmhead_logprob_pkernel<EPI_LOGPROB_NOENT, true, 3> : lmhead_logprob_pkernel<EPI_LOGPROB_NOENT, false, 3>)
                  : cp == 0 ? (ht ? lmhead_logprob_pkernel<EPI_LOGPROB, true, 0> : lmhead_logprob_pkernel<EPI_LOGPROB, false, 0>)
                  : cp == 1 ? (ht ? lmhead_logprob_pkernel<EPI_LOGPROB, true, 1> : lmhead_logprob_pkernel<EPI_LOGPROB, false, 1>)
                  : cp == 2 ? (ht ? lmhead_logprob_pkernel<EPI_LOGPROB, true, 2> : lmhead_logprob_pkernel<EPI_LOGPROB, false, 2>)
                            : (ht ? lmhead_logprob_pkernel<EPI_LOGPROB, true, 3> : lmhead_logprob_pkernel<EPI_LOGPROB, false, 3>);
        hipLaunchKernelGGL(pk, dim3(grid), dim3(512), 0, as_stream(stream), reinterpret_cast<const uint16_t*>(hidden),
                           ld_hidden, reinterpret_cast<const uint16_t*>(weight), ld_weight, T, V, K, mt, nt, group_for(mt),
                           temperature, states, nullptr);
        rc = check_launch("lmhead_logprob_pkernel");
        if (rc) return rc;
        hipLaunchKernelGGL(lmhead_label_merge_kernel, dim3((unsigned)tiles(T, 16)), dim3(64), 0, as_stream(stream),
                           reinterpret_cast<const uint16_t*>(hidden), ld_hidden, reinterpret_cast<const uint16_t*>(weight),
                           ld_weight, T, V, K, labels, label_stride, temperature, temperature != 1.0f ? 1 : 0, states, nt,
                           logp_out, entropy_out, lse_out);
        return check_launch("lmhead_label_merge_kernel");
    }
    const int pipe = pipe_for(T, ld_hidden, V, ld_weight);
    const int bn = tile_n(pipe), mt = tiles(T, BM), nt = tiles(V, bn);
    auto kern = pick_kernel<EPI_LOGPROB>(pipe);
    hipLaunchKernelGGL(kern, dim3(mt * nt), dim3(tile_threads(pipe)), 0, as_stream(stream), reinterpret_cast<const uint16_t*>(hidden),
                       ld_hidden, reinterpret_cast<const uint16_t*>(weight), ld_weight, T, V, K, mt | (group_for(mt) << 16), nullptr, 0ll,
                       temperature, temperature != 1.0f ? 1ull : 0ull, nullptr, 0ll, states, nullptr, nt, labels,
                       label_stride, nullptr);
    rc = check_launch("lmhead_gemm_kernel<logprob>");
    if (rc) return rc;
    return skyrl_lmhead_state_merge(states, nt, T, logp_out, entropy_out, lse_out, stream);
}
