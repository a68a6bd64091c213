// Fused lm_head projection + log-softmax-gather: logprobs of the labels
// straight from the decoder's hidden states, the [N, V] logits never written to HBM.
//
//   lp[n] = h[n]·W[y_n] − logsumexp_v(h[n]·W[v])        h [N, H] bf16, W [V, H] bf16 (nn.Linear)
//
// Replaces `logits = lm_head(hs)` (T5HeadWithValueModel, ppo_models.py:640; GPT lm_head :274,
// :588) followed by logprobs_from_logits (modeling.py:37-41) on the experience side
// (ppo_orchestrator.py:135-155), where no gradient is needed.  Two launches:
//
//   k_lmhead_tiles    MFMA GEMM over 256 x 256 (or 128 x 128) token x vocab tiles (K = H in 64-deep
//                     steps through double-buffered LDS by global_load_lds, 16 B per lane, an
//                     XOR-swizzled image read conflict-free with ds_read_b128); the epilogue
//                     reduces each token's 128 logits of the tile to a partial (max, Σexp)
//                     and the tile that holds the label stores its logit.
//   k_lmhead_combine  one wave per token merges its V/BN partials -> lse, lp = x_y − lse.
//
// The GEMM is MFMA-bound (2·H FLOP per token·vocab pair); the partials cost 8 B per
// (token, vocab tile) — 1/16 of writing the bf16 logits.
#include <type_traits>

#include "common.h"

namespace trlx {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kLmBK = 64;  // K per stage: one 128-B row of bf16 per tile row

// Workgroup tile BM tokens x BN vocab computed by WM x WN waves (each a (BM/WM) x (BN/WN)
// block of 16x16 MFMA tiles).  Two instantiations: 256 x 256 by 8 waves (128 x 64 each: the
// register blocking that keeps the LDS fragment traffic under the MFMA time) for large N,
// 128 x 128 by 4 waves for small batches.
template <int BM_, int BN_, int WM_, int WN_>
struct LmGeom {
    static constexpr int BM = BM_, BN = BN_, WM = WM_, WN = WN_;
    static constexpr int kWaves = WM * WN, kThreads = kWaves * kWave;
    static constexpr int kWRows = BM / WM, kWCols = BN / WN;  // per-wave block
    static constexpr int kMR = kWRows / 16, kNR = kWCols / 16;  // MFMA repeats
    static constexpr int kStage = (BM + BN) * kLmBK * 2;        // A tile + B tile bytes
    static constexpr int kGroupsA = BM / 8, kGroupsB = BN / 8;  // 1-KB glds groups (8 rows)
    static constexpr int kGlds = (kGroupsA + kGroupsB) / kWaves;  // glds per lane per stage
    static constexpr int kLds = 2 * kStage + BM * 4;            // double buffer + labels
    static_assert(kGroupsA % kWaves == 0 && kGroupsB % kWaves == 0, "staging split");
    static_assert(WN * BM * 8 <= 2 * kStage, "combine area");
};
typedef LmGeom<256, 256, 2, 4> LmBig;
typedef LmGeom<128, 128, 2, 2> LmSmall;

struct LmHeadArgs {
    const uint16_t* h;     // [N, H] rows of ldh elements
    const uint16_t* w;     // [V, H] rows of ldw elements
    int64_t ldh, ldw;
    int N, H, V;
    const int64_t* labels; // [N]
    int64_t lb;            // label stride
    float2* part;          // [N, nvt] (max, Σexp) per vocab tile
    float* xlab;           // [N] label logit
    int nvt;
    // a ragged batch (N = B·T tokens, rollouts of T): `rows` = k_ragged_order's list (the valid
    // tokens first, then ~token of the padding), `nrows` its count.  The s2 tiles take token
    // m < *nrows as rows[m] and tiles past the count exit; the combine writes lp = 0 for the
    // padding.  Without rows but with lengths (the other variants): every token computed,
    // the padding's lp written as 0 by the combine.
    const int* rows;
    const int* nrows;
    const int64_t* lengths;
    int T;
};

// Swizzled LDS image of a [rows][64 k] bf16 tile: row r is 128 B; its 16-B chunk c sits at
// physical chunk c ^ ((r >> 1) & 7).  A quarter-wave ds_read_b128 of one chunk column over
// 16 consecutive rows then touches 16 distinct 4-bank groups (even / odd rows fall in the
// two halves of the 256-B bank row): conflict-free.  The map is an involution.
__device__ __forceinline__ int lds_chunk(int r, int c) { return c ^ ((r >> 1) & 7); }

// Stage k-step `kt` of the A (tokens) and B (vocab) tiles: 1-KB wave-instructions of 8 rows;
// lane l lands at LDS slot l of its group (row l>>3, physical chunk l&7) and so fetches the
// logical chunk of that slot.  Rows past N / V are clamped (their results are masked).
template <class G>
__device__ __forceinline__ void lm_stage(const LmHeadArgs& a, char* stage, int m0, int n0, int kt, int wave,
                                         int lane) {
    const int rl = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int i = 0; i < G::kGroupsA / G::kWaves; ++i) {
        const int g = i * G::kWaves + wave;
        const int r = g * 8 + rl;
        const int ma = min(m0 + r, a.N - 1);
        const uint16_t* src = a.h + int64_t(ma) * a.ldh + kt * kLmBK + lds_chunk(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stage + g * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < G::kGroupsB / G::kWaves; ++i) {
        const int g = i * G::kWaves + wave;
        const int r = g * 8 + rl;
        const int nb = min(n0 + r, a.V - 1);
        const uint16_t* src = a.w + int64_t(nb) * a.ldw + kt * kLmBK + lds_chunk(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stage + G::BM * 128 + g * 1024),
                                         16, 0, 0);
    }
}

// All-reduce over each 16-lane DPP row (the 16 columns of a 16x16 MFMA tile row) by four
// row_ror rotations: VALU-latency DPP instead of LDS-latency ds_bpermute chains.  Every lane
// ends with the row's value (the sum's association differs per lane; callers use lane 0).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_max(float v) {
    v = fmaxf(v, dpp_f<0x128>(v));  // row_ror:8
    v = fmaxf(v, dpp_f<0x124>(v));  // row_ror:4
    v = fmaxf(v, dpp_f<0x122>(v));  // row_ror:2
    return fmaxf(v, dpp_f<0x121>(v));  // row_ror:1
}
__device__ __forceinline__ float row16_sum(float v) {
    v += dpp_f<0x128>(v);
    v += dpp_f<0x124>(v);
    v += dpp_f<0x122>(v);
    return v + dpp_f<0x121>(v);
}

__device__ __forceinline__ bf16x8_t lds_frag(const char* tile, int r, int c) {
    return *reinterpret_cast<const bf16x8_t*>(tile + r * 128 + lds_chunk(r, c) * 16);
}

template <class G>
__global__ __launch_bounds__(G::kThreads) void k_lmhead_tiles(LmHeadArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[G::kLds];  // ONE LDS object (glds waits)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / G::WN, wc = wave % G::WN;
    // token tiles fastest: consecutive tiles share the vocab tile (its W rows stay in L2).
    // (An XCD-contiguous remap of blockIdx measured no faster here, round 1: removed.)
    const int ntt = (a.N + G::BM - 1) / G::BM;
    const int b = blockIdx.x;
    const int mt = b % ntt, vt = b / ntt;
    const int m0 = mt * G::BM, n0 = vt * G::BN;
    int* lab = reinterpret_cast<int*>(smem + 2 * G::kStage);
    for (int t = tid; t < G::BM; t += G::kThreads) {
        const int m = m0 + t;
        lab[t] = m < a.N ? int(a.labels[int64_t(m) * a.lb]) : -1;
    }

    f32x4_t acc[G::kMR][G::kNR];
#pragma unroll
    for (int i = 0; i < G::kMR; ++i)
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int nk = a.H / kLmBK;
    lm_stage<G>(a, smem, m0, n0, 0, wave, lane);
    for (int kt = 0; kt < nk; ++kt) {
        const char* cur = smem + (kt & 1) * G::kStage;
        if (kt + 1 < nk) {
            lm_stage<G>(a, smem + ((kt + 1) & 1) * G::kStage, m0, n0, kt + 1, wave, lane);
            // tile kt landed (this wave's part), tile kt+1 stays in flight
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(G::kGlds) : "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();  // ... and every other wave's part too
        const char* At = cur;
        const char* Bt = cur + G::BM * 128;
#pragma unroll
        for (int ks = 0; ks < kLmBK / 32; ++ks) {
            const int c = ks * 4 + (lane >> 4);
            bf16x8_t bfr[G::kNR];
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) bfr[j] = lds_frag(Bt, wc * G::kWCols + j * 16 + (lane & 15), c);
            __builtin_amdgcn_s_setprio(1);  // T5: favour this wave's MFMA issue over the partner's
#pragma unroll
            for (int i = 0; i < G::kMR; ++i) {
                const bf16x8_t af = lds_frag(At, wr * G::kWRows + i * 16 + (lane & 15), c);
#pragma unroll
                for (int j = 0; j < G::kNR; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
            }
            __builtin_amdgcn_s_setprio(0);
        }
        __builtin_amdgcn_s_barrier();  // every wave is done reading `cur` before it is restaged
    }

    // ---- epilogue: per token row, the tile's partial (max, Σexp) and the label logit
    // acc[i][j][q] at lane l = logit(token m0 + wr*kWRows + i*16 + (l>>4)*4 + q,
    //                                 vocab n0 + wc*kWCols + j*16 + (l&15))
    float2* cmb = reinterpret_cast<float2*>(smem);  // [WN][BM], the staging buffers are free now
    const int cl = lane & 15;
#pragma unroll
    for (int i = 0; i < G::kMR; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rt = wr * G::kWRows + i * 16 + (lane >> 4) * 4 + q;  // row in tile
            float x[G::kNR];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) {
                const int v = n0 + wc * G::kWCols + j * 16 + cl;
                x[j] = v < a.V ? acc[i][j][q] : -INFINITY;
                mx = fmaxf(mx, x[j]);
            }
            mx = row16_max(mx);
            // a fully masked row piece (columns >= V) keeps (-inf, 0): exp(-inf - -inf) is NaN
            const float ml2e = mx == -INFINITY ? 0.f : -mx * kLog2e;
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) s += exp2_fast(fmaf(x[j], kLog2e, ml2e));
            s = row16_sum(s);
            if (cl == 0) cmb[wc * G::BM + rt] = make_float2(mx, s);
            const int dy = lab[rt] - (n0 + wc * G::kWCols);
            if (dy >= 0 && dy < G::kWCols && (dy & 15) == cl && m0 + rt < a.N) {
                float xy = x[0];
#pragma unroll
                for (int j = 1; j < G::kNR; ++j) xy = (dy >> 4) == j ? x[j] : xy;
                a.xlab[m0 + rt] = xy;
            }
        }
    }
    __syncthreads();
    for (int t = tid; t < G::BM; t += G::kThreads) {
        if (m0 + t >= a.N) continue;
        float m = -INFINITY;
#pragma unroll
        for (int c = 0; c < G::WN; ++c) m = fmaxf(m, cmb[c * G::BM + t].x);
        float s = 0.f;
        if (m != -INFINITY) {
#pragma unroll
            for (int c = 0; c < G::WN; ++c) {
                const float2 p = cmb[c * G::BM + t];
                s += p.x == -INFINITY ? 0.f : p.y * exp2_fast((p.x - m) * kLog2e);
            }
        }
        a.part[int64_t(m0 + t) * a.nvt + vt] = make_float2(m, s);
    }
}

// ------------------------------------------------------------------ ping-pong, 4 phases per K-step
// 256 x 256 tile, 8 waves (2 x 4, 128 x 64 each) split into two groups by wr.  The waves of
// group 1 start one barrier late, so on every SIMD (one wave of each group) one wave issues
// its LDS reads and LDS-DMA loads while the other runs MFMAs (cdna_hip_programming.md "The
// 256² 8-phase template": ping-pong + counted vmcnt + raw barriers).
//
// A 64-deep K-step is four phases, one per 64 x 32 quadrant (qm, qn) of the wave's block,
// serpentine (0,0) (0,1) (1,1) (1,0) so each phase reads only the operand that changes:
//   q0: A rows qm=0 (8 ds_read_b128) + B cols qn=0 (4)     q1: B cols qn=1 (4)
//   q2: A rows qm=1 (8)                                      q3: nothing (A qm=1, B qn=0 in registers)
// and then issues 16 MFMAs (4 row x 2 col tiles x 2 k-substeps).  LDS holds two K-steps as
// eight 16-KB half-tiles (slot = K-step parity x {HA0, HB0, HB1, HA1}):
//   HA0 = A tile rows {0..63, 128..191}   (qm = 0 of both wave rows)     first read q0
//   HB0 = B tile cols {64·wc + 0..31}     (qn = 0 of the four wave cols)  first read q0
//   HB1 = B tile cols {64·wc + 32..63}                                    first read q1
//   HA1 = A tile rows {64..127, 192..255}                                 first read q2
// Half-tile s (K-step s/4, kind s%4 in that order) is issued (2 LDS DMAs per lane) in phase
// s-6 into the slot of s-8, whose last read was >= 2 phases earlier (WAR), and retired by the
// `vmcnt(8)` of phase s-2 (every phase waits until s <= ph+2), one barrier before its first
// reader (RAW: issuer vmcnt, then a barrier the reader passed).  Four half-tiles stay in flight.
constexpr int kPPHalf = 16384;  // bytes per half-tile: 128 rows x 64 k x 2 B
constexpr int kPPStageBytes = 8 * kPPHalf;
constexpr int kPPLds = kPPStageBytes + LmBig::WN * LmBig::BM * 8 + LmBig::BM * 4;

__device__ __forceinline__ void pp_barrier() { asm volatile("s_barrier" ::: "memory"); }

// Issue half-tile s: 16 groups of 8 rows x 128 B; wave w issues groups w and w + 8.
__device__ __forceinline__ void pp_issue(const LmHeadArgs& a, char* smem, int m0, int n0, int s, int wave, int lane) {
    const int kt = s >> 2, kind = s & 3;
    char* slot = smem + ((kt & 1) * 4 + kind) * kPPHalf;
    const int rl = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int g = i * 8 + wave;
        const int r = g * 8 + rl;  // local row 0..127
        const uint16_t* src;
        if (kind == 0 || kind == 3) {  // A half: tile rows (r>>6)*128 + (kind==3)*64 + (r&63)
            const int tr = (r >> 6) * 128 + (kind == 3 ? 64 : 0) + (r & 63);
            const int ma = min(m0 + tr, a.N - 1);
            src = a.h + int64_t(ma) * a.ldh;
        } else {  // B half: tile cols (r>>5)*64 + (kind==2)*32 + (r&31)
            const int tc = (r >> 5) * 64 + (kind == 2 ? 32 : 0) + (r & 31);
            const int nb = min(n0 + tc, a.V - 1);
            src = a.w + int64_t(nb) * a.ldw;
        }
        src += kt * kLmBK + lds_chunk(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(slot + g * 1024), 16, 0, 0);
    }
}

// ------------------------------------------------------------------ ping-pong, 2 phases per K-step
// As k_lmhead_pingpong with half the barriers: 32 MFMAs per phase (a 64 x 64 half of the
// wave's block).  Phase 2t reads HA0(t), HB0(t), HB1(t) and computes rows qm = 0; phase 2t+1
// reads HA1(t) and computes rows qm = 1.  Stream: phase 2u issues HA0/HB0/HB1 of K-step u+1
// (their slots were last read in phase 2u-2) and waits for HA1(u) (vmcnt(6)); phase 2u+1
// issues HA1(u+1) (slot last read in 2u-1) and waits for K-step u+1's first three (vmcnt(2)).
__global__ __launch_bounds__(512) void k_lmhead_pp2(LmHeadArgs a) {
    typedef LmBig G;
    __shared__ __attribute__((aligned(16))) char smem[kPPLds];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / G::WN, wc = wave % G::WN;
    const int ntt = (a.N + G::BM - 1) / G::BM;
    const int b = blockIdx.x;
    const int mt = b % ntt, vt = b / ntt;
    const int m0 = mt * G::BM, n0 = vt * G::BN;
    float2* cmb = reinterpret_cast<float2*>(smem + kPPStageBytes);
    const int* lab = reinterpret_cast<const int*>(smem + kPPStageBytes + G::WN * G::BM * 8);
    f32x4_t acc[G::kMR][G::kNR];
#pragma unroll
    for (int i = 0; i < G::kMR; ++i)
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int nk = a.H / kLmBK;
    // K-step 0: all four half-tiles; wait for HA0/HB0/HB1 (HA1 may stay in flight)
#pragma unroll
    for (int kind = 0; kind < 4; ++kind) pp_issue(a, smem, m0, n0, kind, wave, lane);
    // labels (low dwords) by LDS DMA behind the operands: no ordinary load (hipcc would wait
    // for it before the first DMA), no latency ahead of K-step 0; read in the epilogue only
    if (wave < 4) {
        const int64_t* src = a.labels + int64_t(min(m0 + wave * 64 + lane, a.N - 1)) * a.lb;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(smem + kPPStageBytes +
                                                                                        G::WN * G::BM * 8 + wave * 256),
                                         4, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // HA0/HB0/HB1 of K-step 0 (HA1 + labels may fly)
    pp_barrier();
    if (wr == 1) pp_barrier();
    bf16x8_t af[2][4];
    bf16x8_t bfr[2][2][2];
    const int fr = lane & 15, fc = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        const char* buf = smem + (kt & 1) * 4 * kPPHalf;
        const bool more = kt + 1 < nk;
        // ---- phase 2kt: rows qm = 0
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i) af[ks][i] = lds_frag(buf, wr * 64 + i * 16 + fr, ks * 4 + fc);
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    bfr[qn][ks][j] = lds_frag(buf + (1 + qn) * kPPHalf, wc * 32 + j * 16 + fr, ks * 4 + fc);
        if (more) {
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 0, wave, lane);
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 1, wave, lane);
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 2, wave, lane);
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // HA1(kt) landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        pp_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int qn = 0; qn < 2; ++qn)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[i][qn * 2 + j] =
                            __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[qn][ks][j], acc[i][qn * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
        // ---- phase 2kt+1: rows qm = 1
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                af[ks][i] = lds_frag(buf + 3 * kPPHalf, wr * 64 + i * 16 + fr, ks * 4 + fc);
        if (more) {
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 3, wave, lane);
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // K-step kt+1's HA0/HB0/HB1 landed
        }
        pp_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int qn = 1; qn >= 0; --qn)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[4 + i][qn * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks][i], bfr[qn][ks][j],
                                                                                        acc[4 + i][qn * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
    }
    if (wr == 0) pp_barrier();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int cl = lane & 15;
#pragma unroll
    for (int i = 0; i < G::kMR; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rt = wr * G::kWRows + i * 16 + (lane >> 4) * 4 + q;
            float x[G::kNR];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) {
                const int v = n0 + wc * G::kWCols + j * 16 + cl;
                x[j] = v < a.V ? acc[i][j][q] : -INFINITY;
                mx = fmaxf(mx, x[j]);
            }
            mx = row16_max(mx);
            const float ml2e = mx == -INFINITY ? 0.f : -mx * kLog2e;
            float sm = 0.f;
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) sm += exp2_fast(fmaf(x[j], kLog2e, ml2e));
            sm = row16_sum(sm);
            if (cl == 0) cmb[wc * G::BM + rt] = make_float2(mx, sm);
            const int dy = lab[rt] - (n0 + wc * G::kWCols);
            if (dy >= 0 && dy < G::kWCols && (dy & 15) == cl && m0 + rt < a.N) {
                float xy = x[0];
#pragma unroll
                for (int j = 1; j < G::kNR; ++j) xy = (dy >> 4) == j ? x[j] : xy;
                a.xlab[m0 + rt] = xy;
            }
        }
    }
    __syncthreads();
    for (int t = tid; t < G::BM; t += G::kThreads) {
        if (m0 + t >= a.N) continue;
        float m = -INFINITY;
#pragma unroll
        for (int c = 0; c < G::WN; ++c) m = fmaxf(m, cmb[c * G::BM + t].x);
        float sm = 0.f;
        if (m != -INFINITY) {
#pragma unroll
            for (int c = 0; c < G::WN; ++c) {
                const float2 p = cmb[c * G::BM + t];
                sm += p.x == -INFINITY ? 0.f : p.y * exp2_fast((p.x - m) * kLog2e);
            }
        }
        a.part[int64_t(m0 + t) * a.nvt + vt] = make_float2(m, sm);
    }
}

// ------------------------------------------------------------------ two workgroups per CU
// 128 tokens x 256 vocab per workgroup of 4 waves (2 x 2, 64 x 128 each, one wave per SIMD),
// K in 32-deep steps through a 3-slot LDS ring (24 KB per step: 64-B rows, chunk-XOR
// swizzled), ONE raw barrier per step, the next step's fragments read into a second register
// set while this step's 32 MFMAs run.  74.5 KB of LDS and <= 256 VGPRs let TWO workgroups
// share a CU, on different tiles and phases: while one runs its barrier or its per-tile
// log-sum-exp epilogue (~1,300 VALU per wave), the other's wave on the same SIMD issues MFMAs
// — the epilogue no longer idles the MFMA pipe as in k_lmhead_pp2, whose two waves per SIMD
// belong to one tile.
constexpr int kS2BK = 32;
constexpr int kS2Stage = (128 + 256) * kS2BK * 2;  // 24 KB: A 128 rows + B 256 rows of 64 B
constexpr int kS2Lds = 3 * kS2Stage + 2 * 128 * 8 + 128 * 4;
typedef LmGeom<128, 256, 2, 2> LmS2;
static_assert(LmS2::kMR == 4 && LmS2::kNR == 8, "s2 wave block is 64 x 128");

// 64-B rows: physical 16-B chunk c ^ ((r >> 2) & 3) (a quarter-wave ds_read_b128 of one
// logical chunk over 16 consecutive rows then covers all 64 banks once).
__device__ __forceinline__ int s2_chunk(int r, int c) { return c ^ ((r >> 2) & 3); }
__device__ __forceinline__ bf16x8_t s2_frag(const char* tile, int r, int c) {
    return *reinterpret_cast<const bf16x8_t*>(tile + r * 64 + s2_chunk(r, c) * 16);
}

// RAGGED: token m of the tile grid is row rows[m] of a ragged batch, m < *nrows (the valid
// tokens, k_ragged_order); tiles past the count exit at once, so padding costs no MFMA work.
template <bool RAGGED>
__global__ __launch_bounds__(256, 2) void k_lmhead_s2(LmHeadArgs a) {
    typedef LmS2 G;
    __shared__ __attribute__((aligned(16))) char smem[kS2Lds];  // ONE LDS object (glds waits)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    const int nv = RAGGED ? *a.nrows : a.N;  // tokens of the grid (block-uniform)
    if (RAGGED && nv == 0) return;
    // token tiles fastest (the weight tile stays in L2 across them); ragged: over the valid
    // tokens' tiles only, so the grid's surplus blocks are its last ones (they exit at once —
    // interleaved with working ones they would idle CU slots, vocab_rows.hip k_ragged_order)
    const int ntt = ((RAGGED ? nv : a.N) + G::BM - 1) / G::BM;
    const int b = blockIdx.x;
    const int mt = b % ntt, vt = b / ntt;
    if (RAGGED && vt >= a.nvt) return;
    const int m0 = mt * G::BM, n0 = vt * G::BN;
    float2* cmb = reinterpret_cast<float2*>(smem + 3 * kS2Stage);
    int* lab = reinterpret_cast<int*>(smem + 3 * kS2Stage + 2 * G::BM * 8);
    if (tid < G::BM) {  // before any LDS DMA: an ordinary load later would drain them (vmcnt(0))
        const int m = m0 + tid;
        lab[tid] = m < nv ? int(a.labels[int64_t(RAGGED ? a.rows[m] : m) * a.lb]) : -1;
    }
    // DMA groups: 16 rows x 64 B per wave instruction; groups 0..7 = the A tile (tokens),
    // 8..23 = the B tile (vocab); wave w issues groups w, w+4, ..., w+20.  Lane l -> row
    // l >> 2, physical chunk l & 3, fetching the logical chunk s2_chunk(row, physical).
    // Buffer resources on the tile bases: the per-lane row offset (rows clamped to the last
    // valid one) stays in VOFFSET for the whole K loop, the K step rides SOFFSET: no VALU per
    // DMA.
    const int rl = lane >> 2;
    const int lc = (lane & 3) ^ ((lane >> 4) & 3);
    // (RAGGED: the A rows are gathered — the resource starts at token 0, each lane's offset
    // is its token's row; the host checks N·ldh·2 < 2^31)
    const __amdgpu_buffer_rsrc_t rA = make_rsrc(a.h + (RAGGED ? int64_t(0) : int64_t(m0) * a.ldh), 0x7ffffff0u);
    const __amdgpu_buffer_rsrc_t rB = make_rsrc(a.w + int64_t(n0) * a.ldw, 0x7ffffff0u);
    int voff[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int g = i * 4 + wave;
        if (i < 2) {
            const int r = min(g * 16 + rl, nv - 1 - m0);
            const int row = RAGGED ? a.rows[m0 + r] : r;
            voff[i] = (row * int(a.ldh) + lc * 8) * 2;
        } else {
            const int r = min((g - 8) * 16 + rl, a.V - 1 - n0);
            voff[i] = (r * int(a.ldw) + lc * 8) * 2;
        }
    }
    auto issue = [&](int kt) {
        char* stage = smem + (kt % 3) * kS2Stage;
        const int soff = kt * kS2BK * 2;
#pragma unroll
        for (int i = 0; i < 6; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                i < 2 ? rA : rB, (__attribute__((address_space(3))) void*)(stage + (i * 4 + wave) * 1024), 16,
                voff[i], soff, 0, 0);
    };
    f32x4_t acc[G::kMR][G::kNR];
#pragma unroll
    for (int i = 0; i < G::kMR; ++i)
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fc = lane >> 4;
    // K loop, one raw barrier per 32-deep step: retire step kt (own vmcnt, leaving kt+1 in
    // flight; then the barrier: every wave's part landed AND every wave is done reading kt-1),
    // issue the DMA of kt+2 into kt-1's slot, read kt's fragments, 32 MFMAs.  The second
    // workgroup on the CU fills this wave's barrier and LDS-latency gaps.
    const int nk = a.H / kS2BK;
    issue(0);
    if (nk > 1) issue(1);
    for (int kt = 0; kt < nk; ++kt) {
        if (kt + 1 < nk)
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (kt + 2 < nk) issue(kt + 2);
        const char* At = smem + (kt % 3) * kS2Stage;
        const char* Bt = At + G::BM * 64;
        bf16x8_t af[G::kMR], bfr[G::kNR];
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) bfr[j] = s2_frag(Bt, wc * G::kWCols + j * 16 + fr, fc);
#pragma unroll
        for (int i = 0; i < G::kMR; ++i) af[i] = s2_frag(At, wr * G::kWRows + i * 16 + fr, fc);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < G::kMR; ++i)
#pragma unroll
            for (int j = 0; j < G::kNR; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();  // the labels' LDS writes (before the loop) and the stages are done with

    // ---- epilogue (as k_lmhead_tiles): per token row, the tile's partial (max, Σexp) and
    // the label logit; acc[i][j][q] at lane l = logit(token m0 + wr*64 + i*16 + (l>>4)*4 + q,
    // vocab n0 + wc*128 + j*16 + (l&15))
    const int cl = lane & 15;
#pragma unroll
    for (int i = 0; i < G::kMR; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rt = wr * G::kWRows + i * 16 + (lane >> 4) * 4 + q;
            float x[G::kNR];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) {
                const int v = n0 + wc * G::kWCols + j * 16 + cl;
                x[j] = v < a.V ? acc[i][j][q] : -INFINITY;
                mx = fmaxf(mx, x[j]);
            }
            mx = row16_max(mx);
            const float ml2e = mx == -INFINITY ? 0.f : -mx * kLog2e;
            float sm = 0.f;
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) sm += exp2_fast(fmaf(x[j], kLog2e, ml2e));
            sm = row16_sum(sm);
            if (cl == 0) cmb[wc * G::BM + rt] = make_float2(mx, sm);
            const int dy = lab[rt] - (n0 + wc * G::kWCols);
            if (dy >= 0 && dy < G::kWCols && (dy & 15) == cl && m0 + rt < nv) {
                float xy = x[0];
#pragma unroll
                for (int j = 1; j < G::kNR; ++j) xy = (dy >> 4) == j ? x[j] : xy;
                a.xlab[m0 + rt] = xy;
            }
        }
    }
    __syncthreads();
    for (int t = tid; t < G::BM; t += G::kThreads) {
        if (m0 + t >= nv) continue;
        float m = -INFINITY;
#pragma unroll
        for (int c = 0; c < G::WN; ++c) m = fmaxf(m, cmb[c * G::BM + t].x);
        float sm = 0.f;
        if (m != -INFINITY) {
#pragma unroll
            for (int c = 0; c < G::WN; ++c) {
                const float2 p = cmb[c * G::BM + t];
                sm += p.x == -INFINITY ? 0.f : p.y * exp2_fast((p.x - m) * kLog2e);
            }
        }
        a.part[int64_t(m0 + t) * a.nvt + vt] = make_float2(m, sm);
    }
}

// One wave per token: merge the nvt partials (fixed order per lane, then a fixed butterfly).
__global__ __launch_bounds__(256) void k_lmhead_combine(LmHeadArgs a, void* lp, int lp_dtype, float* lse_out) {
    const int lane = threadIdx.x & 63;
    const int64_t n = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);  // partials index
    if (n >= a.N) return;
    int64_t tok = n;  // output token
    bool pad = false;
    if (a.rows) {  // compact index n: valid token rows[n], or the padding token ~rows[n]
        const int r = a.rows[n];
        pad = n >= *a.nrows;
        tok = pad ? ~int64_t(r) : int64_t(r);
    } else if (a.lengths) {
        pad = n % a.T >= a.lengths[n / a.T];
    }
    if (pad) {  // the padded store's 0.0 (ppo_pipeline.py:47-65)
        if (lane == 0) {
            st_any(lp, lp_dtype, tok, 0.0f);
            if (lse_out) lse_out[tok] = 0.0f;
        }
        return;
    }
    const float2* p = a.part + n * a.nvt;
    float m = -INFINITY, s = 0.f;
    for (int t = lane; t < a.nvt; t += kWave) {
        const float2 q = p[t];
        if (q.x == -INFINITY) continue;
        const float nm = fmaxf(m, q.x);
        s = (m == -INFINITY ? 0.f : s * exp2_fast((m - nm) * kLog2e)) + q.y * exp2_fast((q.x - nm) * kLog2e);
        m = nm;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const float m2 = __shfl_xor(m, off, kWave), s2 = __shfl_xor(s, off, kWave);
        const float nm = fmaxf(m, m2);
        if (nm != -INFINITY)
            s = (m == -INFINITY ? 0.f : s * exp2_fast((m - nm) * kLog2e)) +
                (m2 == -INFINITY ? 0.f : s2 * exp2_fast((m2 - nm) * kLog2e));
        m = nm;
    }
    const int64_t y = a.labels[tok * a.lb];
    const bool y_ok = y >= 0 && y < a.V;
    if (lane == 0) {
        const float lse = m + logf(s);
        const float lpv = y_ok ? a.xlab[n] - lse : NAN;  // label logit picked out by the tile kernel
        st_any(lp, lp_dtype, tok, lpv);
        if (lse_out) lse_out[tok] = lse;
    }
}

}  // namespace trlx

using namespace trlx;

// variant: 0 auto, 3 128x128 tiles (k_lmhead_tiles<LmSmall>), 8 256x256 ping-pong with 2 phases
// per K-step (k_lmhead_pp2).  auto (measured on MI355X, tools/lmhead_bench.py, interleaved
// rounds): N >= 2048 -> 8 (1.1-1.4x the 2-barrier 256x256 tiles at every BASELINE shape);
// small N -> 128x128 tiles (enough workgroups to fill 256 CUs).  Round 1 also measured a
// persistent 3-stage form, a 4-phase ping-pong (with and without an XCD remap), persistent
// ping-pongs and a 32-deep 4-slot ring: all slower than or tied with variant 8;
// they were removed from the library in round 2 (git history: lmhead_rows.hip at 63d22a9).
// Round 3: 9 = 128 x 256 tiles, two workgroups per CU (k_lmhead_s2): 0.95x variant 8 at C2's
// H = 768 (519 vs 544 us), tied at C3, 1.23x slower at H = 4096 (its 32-deep 3-slot ring
// keeps only ~2 K-steps of DMA in flight; profiles/r03_lmhead_s2_bench.log) -> auto for H <= 1024.
static TuneKnob g_lm_variant{0};
static int lm_variant(int64_t N, int64_t H) {
    if (g_lm_variant) return g_lm_variant;
    return N < 2048 ? 3 : (H <= 1024 ? 9 : 8);
}
static int lm_tile_n(int64_t N, int64_t H) { return lm_variant(N, H) == 3 ? LmSmall::BN : LmBig::BN; }  // s2: 256
static_assert(LmSmall::BN == 128 && LmBig::BN == 256, "tile widths");

extern "C" int trlx_lmhead_set_variant(int v) {
    TRLX_REQUIRE(v == 0 || v == 3 || v == 8 || v == 9, TRLX_ERR_ARG, "lmhead variant must be 0 (auto), 3, 8 or 9");
    g_lm_variant = v;
    return TRLX_OK;
}

extern "C" int64_t trlx_lmhead_workspace_bytes(int64_t N, int64_t V) {
    const int64_t nvt = (V + lm_tile_n(N, 0) - 1) / lm_tile_n(N, 0);  // every N >= 2048 variant has BN = 256
    return N * nvt * int64_t(sizeof(float2)) + N * int64_t(sizeof(float));
}

static int lm_launch_small(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntt = (a.N + LmSmall::BM - 1) / LmSmall::BM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    hipLaunchKernelGGL((k_lmhead_tiles<LmSmall>), dim3(unsigned(ntt * a.nvt)), dim3(LmSmall::kThreads), 0, stream,
                       a);
    return check_launch("k_lmhead_tiles");
}

static int lm_launch_s2(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntt = (a.N + LmS2::BM - 1) / LmS2::BM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    TRLX_REQUIRE(a.H % kS2BK == 0, TRLX_ERR_SHAPE, "hidden size must be a multiple of %d", kS2BK);
    if (a.rows)
        hipLaunchKernelGGL(k_lmhead_s2<true>, dim3(unsigned(ntt * a.nvt)), dim3(256), 0, stream, a);
    else
        hipLaunchKernelGGL(k_lmhead_s2<false>, dim3(unsigned(ntt * a.nvt)), dim3(256), 0, stream, a);
    return check_launch("k_lmhead_s2");
}

static int lm_launch_pp2(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntt = (a.N + LmBig::BM - 1) / LmBig::BM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    hipLaunchKernelGGL(k_lmhead_pp2, dim3(unsigned(ntt * a.nvt)), dim3(512), 0, stream, a);
    return check_launch("k_lmhead_pp2");
}

static int lmhead_impl(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N, int64_t H,
                       int64_t V, const int64_t* labels, int64_t lb, const int64_t* lengths, int64_t T, void* order_ws,
                       void* lp_out, int lp_dtype, float* lse_out, void* workspace, void* stream) {
    TRLX_REQUIRE(hidden && weight && labels && lp_out && workspace, TRLX_ERR_ARG, "NULL argument");
    TRLX_REQUIRE(N >= 0 && V > 0 && H > 0, TRLX_ERR_SHAPE, "bad shape N=%lld H=%lld V=%lld", (long long)N,
                 (long long)H, (long long)V);
    TRLX_REQUIRE(H % kLmBK == 0, TRLX_ERR_SHAPE, "hidden size %lld must be a multiple of %d", (long long)H, kLmBK);
    TRLX_REQUIRE(ldh % 8 == 0 && ldw % 8 == 0 && ldh >= H && ldw >= H, TRLX_ERR_STRIDE,
                 "row strides must be >= H and multiples of 8 elements (16-B rows)");
    TRLX_REQUIRE((reinterpret_cast<uintptr_t>(hidden) & 15) == 0 && (reinterpret_cast<uintptr_t>(weight) & 15) == 0,
                 TRLX_ERR_STRIDE, "hidden / weight must be 16-B aligned");
    TRLX_REQUIRE(N < (int64_t(1) << 31) && V < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too large");
    TRLX_REQUIRE(lp_dtype == TRLX_F32 || lp_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "lp dtype");
    if (N == 0) return TRLX_OK;
    LmHeadArgs a = {};
    a.h = static_cast<const uint16_t*>(hidden);
    a.w = static_cast<const uint16_t*>(weight);
    a.ldh = ldh;
    a.ldw = ldw;
    a.N = int(N);
    a.H = int(H);
    a.V = int(V);
    a.labels = labels;
    a.lb = lb;
    const int bn = lm_tile_n(N, H);
    a.nvt = int((V + bn - 1) / bn);
    a.part = static_cast<float2*>(workspace);
    a.xlab = reinterpret_cast<float*>(static_cast<char*>(workspace) + N * a.nvt * int64_t(sizeof(float2)));
    const int var = lm_variant(N, H);
    if (lengths) {
        TRLX_REQUIRE(T > 0 && N % T == 0, TRLX_ERR_SHAPE, "ragged lm_head: N = %lld is not B x T = %lld",
                     (long long)N, (long long)T);
        a.lengths = lengths;
        a.T = int(T);
        if (var == 9 && order_ws) {  // the s2 tiles take the valid tokens only
            TRLX_REQUIRE(N * ldh * 2 < (int64_t(1) << 31), TRLX_ERR_SHAPE, "ragged lm_head: hidden rows span >= 2 GB");
            const int orc = launch_ragged_order(lengths, N / T, T, static_cast<int*>(order_ws), (hipStream_t)stream);
            if (orc) return orc;
            a.rows = static_cast<const int*>(order_ws);
            a.nrows = a.rows + N;
        }
    }
    const int rc = var == 8   ? lm_launch_pp2(a, (hipStream_t)stream)
                   : var == 9 ? lm_launch_s2(a, (hipStream_t)stream)
                              : lm_launch_small(a, (hipStream_t)stream);
    if (rc) return rc;
    hipLaunchKernelGGL(k_lmhead_combine, dim3(unsigned((N + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a, lp_out,
                       lp_dtype, lse_out);
    return check_launch("k_lmhead_combine");
}

extern "C" int trlx_lmhead_logprobs(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                    int64_t H, int64_t V, const int64_t* labels, int64_t lb, void* lp_out,
                                    int lp_dtype, float* lse_out, void* workspace, void* stream) {
    return lmhead_impl(hidden, ldh, weight, ldw, N, H, V, labels, lb, nullptr, 0, nullptr, lp_out, lp_dtype, lse_out,
                       workspace, stream);
}

extern "C" int trlx_lmhead_logprobs_ragged(const void* hidden, int64_t ldh, const void* weight, int64_t ldw,
                                           int64_t N, int64_t H, int64_t V, const int64_t* labels, int64_t lb,
                                           const int64_t* lengths, int64_t T, void* order_ws, void* lp_out,
                                           int lp_dtype, float* lse_out, void* workspace, void* stream) {
    return lmhead_impl(hidden, ldh, weight, ldw, N, H, V, labels, lb, lengths, T, order_ws, lp_out, lp_dtype, lse_out,
                       workspace, stream);
}
