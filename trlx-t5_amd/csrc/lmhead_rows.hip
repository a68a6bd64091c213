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
    int xcd_swizzle;       // 1: remap blockIdx so each XCD gets a contiguous range of tiles
    int dbg;               // ping-pong ablation bits (timing probes only; 0 = normal)
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
    // Workgroups are dealt round-robin to the 8 XCDs; with xcd_swizzle each XCD's share is a
    // contiguous tile range (bijective remap, cdna_hip_programming.md T1) — speed only.
    const int ntt = (a.N + G::BM - 1) / G::BM;
    int b = blockIdx.x;
    if (a.xcd_swizzle) {
        const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = b % 8;
        b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    }
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

// ------------------------------------------------------------------ persistent, 3 stages in flight
// One workgroup per CU walks its tiles (blockIdx.x, +gridDim.x, ...) as ONE stream of 32-deep
// K-steps: four LDS stages, three in flight, and the stream runs straight across tile
// boundaries — the next tile's first stages load while the current tile's epilogue runs, so
// no tile pays the operand-fetch latency up front (at H = 768 a tile is only 24 K-steps).
// One barrier per step: the wait for stage s, then the barrier that both publishes it and
// frees stage s-1's buffer for the load of step s+3.  Every load of the loop is an LDS DMA
// (an ordinary load would make hipcc drain the queue); the label logit is not picked out
// here but recomputed by the combine kernel as one H-long dot product per token.
constexpr int kPBK = 32;      // K per stage: 64-B rows
constexpr int kPStages = 4;

template <class G>
struct LmPersist {
    static constexpr int kStage = (G::BM + G::BN) * kPBK * 2;
    static constexpr int kGroupsA = G::BM / 16, kGroupsB = G::BN / 16;  // 1-KB groups: 16 rows x 64 B
    static constexpr int kGlds = (kGroupsA + kGroupsB) / G::kWaves;
    static constexpr int kCmbOff = kPStages * kStage;
    static constexpr int kLds = kCmbOff + G::WN * G::BM * 8;
    static_assert(kGroupsA % G::kWaves == 0 && kGroupsB % G::kWaves == 0, "staging split");
};

// 64-B rows: chunk c of row r sits at c ^ ((r >> 2) & 3); the 16 rows a quarter-wave reads
// then cover the 64 banks exactly once.
__device__ __forceinline__ int lds_chunk64(int r, int c) { return c ^ ((r >> 2) & 3); }

__device__ __forceinline__ bf16x8_t lds_frag64(const char* tile, int r, int c) {
    return *reinterpret_cast<const bf16x8_t*>(tile + r * 64 + lds_chunk64(r, c) * 16);
}

template <class G>
__device__ __forceinline__ void lmp_stage(const LmHeadArgs& a, char* stage, int m0, int n0, int kt, int wave,
                                          int lane) {
    typedef LmPersist<G> P;
    const int rl = lane >> 2, pc = lane & 3;
#pragma unroll
    for (int i = 0; i < P::kGroupsA / G::kWaves; ++i) {
        const int g = i * G::kWaves + wave;
        const int r = g * 16 + rl;
        const int ma = min(m0 + r, a.N - 1);
        const uint16_t* src = a.h + int64_t(ma) * a.ldh + kt * kPBK + lds_chunk64(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stage + g * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < P::kGroupsB / G::kWaves; ++i) {
        const int g = i * G::kWaves + wave;
        const int r = g * 16 + rl;
        const int nb = min(n0 + r, a.V - 1);
        const uint16_t* src = a.w + int64_t(nb) * a.ldw + kt * kPBK + lds_chunk64(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(stage + G::BM * 64 + g * 1024),
                                         16, 0, 0);
    }
}

// An LDS store hipcc cannot see: a plain ds_write while LDS DMAs are in flight makes hipcc
// wait vmcnt(0) first (it cannot prove the addresses differ), which would drain the three
// stages in flight at every tile epilogue.  The combine area never overlaps a stage buffer.
__device__ __forceinline__ void lds_store_f2(float2* p, float x, float y) {
    const uint32_t addr = uint32_t(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) float2*)p));
    asm volatile("ds_write_b64 %0, %1" ::"v"(addr), "v"(make_float2(x, y)) : "memory");
}

__device__ __forceinline__ float2 lds_load_f2(const float2* p) {
    const uint32_t addr = uint32_t(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const float2*)p));
    float2 v;
    asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

// s_waitcnt vmcnt(n) for the wave-uniform n of the pipeline (n in {0, g, 2g}).
template <int GL>
__device__ __forceinline__ void lmp_wait(int n) {
    if (n == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (n == GL) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GL) : "memory");
    else asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GL) : "memory");
}

template <class G>
__global__ __launch_bounds__(G::kThreads) void k_lmhead_persist(LmHeadArgs a, int ntiles) {
    typedef LmPersist<G> P;
    __shared__ __attribute__((aligned(16))) char smem[P::kLds];  // ONE LDS object (glds waits)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / G::WN, wc = wave % G::WN;
    const int ntt = (a.N + G::BM - 1) / G::BM;
    const int nk = a.H / kPBK;
    const int mine = (ntiles - int(blockIdx.x) + int(gridDim.x) - 1) / int(gridDim.x);
    if (mine <= 0) return;
    const int S = mine * nk;
    float2* cmb = reinterpret_cast<float2*>(smem + P::kCmbOff);

    auto loads_of = [&](int x) { return x >= S ? 0 : P::kGlds; };
    auto issue = [&](int x) {
        const int j = x / nk, kt = x - j * nk;
        const int t = int(blockIdx.x) + j * int(gridDim.x);
        const int mt = t % ntt, vt = t / ntt;
        lmp_stage<G>(a, smem + (x % kPStages) * P::kStage, mt * G::BM, vt * G::BN, kt, wave, lane);
    };

    f32x4_t acc[G::kMR][G::kNR];
#pragma unroll
    for (int i = 0; i < G::kMR; ++i)
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int x = 0; x < 3 && x < S; ++x) issue(x);
    for (int s = 0; s < S; ++s) {
        lmp_wait<P::kGlds>(loads_of(s + 1) + loads_of(s + 2));  // stage s landed (this wave's part)
        __builtin_amdgcn_s_barrier();  // ... every wave's part; and stage s-1's buffer is free
        if (s + 3 < S) issue(s + 3);
        const char* At = smem + (s % kPStages) * P::kStage;
        const char* Bt = At + G::BM * 64;
        const int c = lane >> 4;
        bf16x8_t bfr[G::kNR];
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) bfr[j] = lds_frag64(Bt, wc * G::kWCols + j * 16 + (lane & 15), c);
#pragma unroll
        for (int i = 0; i < G::kMR; ++i) {
            const bf16x8_t af = lds_frag64(At, wr * G::kWRows + i * 16 + (lane & 15), c);
#pragma unroll
            for (int j = 0; j < G::kNR; ++j)
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
        }
        if (s % nk != nk - 1) continue;

        // ---- tile epilogue (as k_lmhead_tiles), raw barriers: a __syncthreads() would drain
        // the stages in flight
        const int jt = s / nk;
        const int t = int(blockIdx.x) + jt * int(gridDim.x);
        const int m0 = (t % ntt) * G::BM, vt = t / ntt, n0 = vt * G::BN;
        const int cl = lane & 15;
#pragma unroll
        for (int i = 0; i < G::kMR; ++i) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rt = wr * G::kWRows + i * 16 + (lane >> 4) * 4 + q;
                float xv[G::kNR];
                float mx = -INFINITY;
#pragma unroll
                for (int j = 0; j < G::kNR; ++j) {
                    const int v = n0 + wc * G::kWCols + j * 16 + cl;
                    xv[j] = v < a.V ? acc[i][j][q] : -INFINITY;
                    mx = fmaxf(mx, xv[j]);
                }
                mx = row16_max(mx);
                const float ml2e = mx == -INFINITY ? 0.f : -mx * kLog2e;
                float sm = 0.f;
#pragma unroll
                for (int j = 0; j < G::kNR; ++j) sm += exp2_fast(fmaf(xv[j], kLog2e, ml2e));
                sm = row16_sum(sm);
                if (cl == 0) lds_store_f2(cmb + wc * G::BM + rt, mx, sm);
            }
        }
#pragma unroll
        for (int i = 0; i < G::kMR; ++i)
#pragma unroll
            for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        for (int r = tid; r < G::BM; r += G::kThreads) {
            if (m0 + r >= a.N) continue;
            float2 pw[G::WN];
            float m = -INFINITY;
#pragma unroll
            for (int c2 = 0; c2 < G::WN; ++c2) {
                pw[c2] = lds_load_f2(cmb + c2 * G::BM + r);
                m = fmaxf(m, pw[c2].x);
            }
            float sm = 0.f;
            if (m != -INFINITY) {
#pragma unroll
                for (int c2 = 0; c2 < G::WN; ++c2)
                    sm += pw[c2].x == -INFINITY ? 0.f : pw[c2].y * exp2_fast((pw[c2].x - m) * kLog2e);
            }
            a.part[int64_t(m0 + r) * a.nvt + vt] = make_float2(m, sm);
        }
        // the next tile's epilogue rewrites cmb only after many barriers
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

// vmcnt(2n) for the wave-uniform n in [0, 4]
__device__ __forceinline__ void pp_wait(int n) {
    switch (n) {
        case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
        case 1: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
        case 2: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
        case 3: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
        default: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    }
}

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

__global__ __launch_bounds__(512) void k_lmhead_pingpong(LmHeadArgs a) {
    typedef LmBig G;
    __shared__ __attribute__((aligned(16))) char smem[kPPLds];  // ONE LDS object (glds waits)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / G::WN, wc = wave % G::WN;
    const int ntt = (a.N + G::BM - 1) / G::BM;
    int b = blockIdx.x;
    if (a.xcd_swizzle) {
        const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = b % 8;
        b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    }
    const int mt = b % ntt, vt = b / ntt;
    const int m0 = mt * G::BM, n0 = vt * G::BN;
    float2* cmb = reinterpret_cast<float2*>(smem + kPPStageBytes);
    int* lab = reinterpret_cast<int*>(smem + kPPStageBytes + G::WN * G::BM * 8);
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
    const int S = 4 * nk;
    const int pro = S < 6 ? S : 6;
    for (int s = 0; s < pro; ++s) pp_issue(a, smem, m0, n0, s, wave, lane);
    pp_wait(min(4, (pro - 2) > 0 ? pro - 2 : 0));  // half-tiles 0, 1 (K-step 0's q0 operands) retired
    pp_barrier();  // raw: __syncthreads() would drain the prefetch (lab[] is read after many barriers)
    if (wr == 1) pp_barrier();                    // group 1 runs one barrier behind

    bf16x8_t af[2][4];     // A fragments of the current qm: [k-substep][row tile]
    bf16x8_t bfr[2][2][2]; // B fragments: [qn][k-substep][col tile]
    const int fr = lane & 15, fc = lane >> 4;
    // One phase of the stream; STEADY: the half-tile issue is in range and vmcnt(8) is exact
    // (every K-step but the last two), so the body has no bounds logic.
    auto phase = [&](int kt, auto qc, auto steadyc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        constexpr bool steady = decltype(steadyc)::value;
        const char* buf = smem + (kt & 1) * 4 * kPPHalf;
        const int ph = 4 * kt + q;
        // ---- memory section: fragments of this phase, then one half-tile of the stream
        if constexpr (q == 0 || q == 2) {
            if (!(a.dbg & 4)) {
                const char* At = buf + (q == 0 ? 0 : 3) * kPPHalf;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int i = 0; i < 4; ++i) af[ks][i] = lds_frag(At, wr * 64 + i * 16 + fr, ks * 4 + fc);
            }
        }
        if constexpr (q == 0 || q == 1) {
            if (!(a.dbg & 4)) {
                const char* Bt = buf + (q == 0 ? 1 : 2) * kPPHalf;
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int j = 0; j < 2; ++j) bfr[q][ks][j] = lds_frag(Bt, wc * 32 + j * 16 + fr, ks * 4 + fc);
            }
        }
        if constexpr (steady) {
            if (!(a.dbg & 2)) pp_issue(a, smem, m0, n0, ph + 6, wave, lane);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            if (ph + 6 < S && !(a.dbg & 2)) pp_issue(a, smem, m0, n0, ph + 6, wave, lane);
            const int n = min(ph + 6, S - 1) - (ph + 2);
            pp_wait(n < 0 ? 0 : (n > 4 ? 4 : n));
        }
        pp_barrier();
        // ---- MFMA section: quadrant (qm, qn) = (0,0) (0,1) (1,1) (1,0)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        constexpr int qm = q >= 2 ? 1 : 0;
        constexpr int qn = (q == 1 || q == 2) ? 1 : 0;
        __builtin_amdgcn_s_setprio(1);
        if (!(a.dbg & 1)) {
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j < 2; ++j)
                        acc[qm * 4 + i][qn * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                            af[ks][i], bfr[qn][ks][j], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
    };
    typedef std::integral_constant<bool, true> Steady;
    typedef std::integral_constant<bool, false> Tail;
    int kt = 0;
    for (; kt + 2 < nk; ++kt) {
        phase(kt, std::integral_constant<int, 0>{}, Steady{});
        phase(kt, std::integral_constant<int, 1>{}, Steady{});
        phase(kt, std::integral_constant<int, 2>{}, Steady{});
        phase(kt, std::integral_constant<int, 3>{}, Steady{});
    }
    for (; kt < nk; ++kt) {
        phase(kt, std::integral_constant<int, 0>{}, Tail{});
        phase(kt, std::integral_constant<int, 1>{}, Tail{});
        phase(kt, std::integral_constant<int, 2>{}, Tail{});
        phase(kt, std::integral_constant<int, 3>{}, Tail{});
    }
    if (wr == 0) pp_barrier();  // balance group 1's extra barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- epilogue (as k_lmhead_tiles): per token row, the tile's partial (max, Σexp) and
    // the label logit.  acc[I][J][r] at lane l = logit(token m0 + wr*128 + I*16 + (l>>4)*4 + r,
    //                                             vocab n0 + wc*64 + J*16 + (l&15))
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
    int b = blockIdx.x;
    if (a.xcd_swizzle) {
        const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = b % 8;
        b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    }
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
    if ((a.dbg & 8) && wr == 1) __builtin_amdgcn_s_setprio(1);  // static priority for the younger half
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
        if (more && !(a.dbg & 2)) {
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 0, wave, lane);
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 1, wave, lane);
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 2, wave, lane);
            asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // HA1(kt) landed
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        pp_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (!(a.dbg & 24)) __builtin_amdgcn_s_setprio(1);
        if (!(a.dbg & 1))
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
        if (!(a.dbg & 24)) __builtin_amdgcn_s_setprio(0);
        pp_barrier();
        // ---- phase 2kt+1: rows qm = 1
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                af[ks][i] = lds_frag(buf + 3 * kPPHalf, wr * 64 + i * 16 + fr, ks * 4 + fc);
        if (more && !(a.dbg & 2)) {
            pp_issue(a, smem, m0, n0, 4 * (kt + 1) + 3, wave, lane);
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // K-step kt+1's HA0/HB0/HB1 landed
        }
        pp_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (!(a.dbg & 24)) __builtin_amdgcn_s_setprio(1);
        if (!(a.dbg & 1))
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
        if (!(a.dbg & 24)) __builtin_amdgcn_s_setprio(0);
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

// ------------------------------------------------------------------ ping-pong, 32-deep K-steps, 4-slot ring
// The 2-phase schedule's MFMA : barrier ratio with a deeper operand stream: a K-step is 32
// deep (32 KB of A + B), LDS holds a ring of four, and each phase consumes one K-step with
// 32 MFMAs per wave (12 fragment reads: 8 A row tiles, 4 B column tiles).  Phase t issues
// K-step t+3 into the slot of t-1 and waits (vmcnt(8)) for K-step t+1, so every operand has
// two phases to land.  WAR: the reading group retires its fragment reads (lgkmcnt(0)) before
// the barrier that ends its memory section, so a slot is free for DMA right after it.
constexpr int kP9BK = 32;
constexpr int kP9Slot = (LmBig::BM + LmBig::BN) * kP9BK * 2;  // 32 KB
constexpr int kP9LabOff = 4 * kP9Slot + LmBig::WN * LmBig::BM * 8;
constexpr int kP9Lds = kP9LabOff + LmBig::BM * 4;

// K-step kt (32 deep) -> ring slot kt & 3: A then B, 1-KB groups of 16 rows x 64 B; wave w
// issues A groups w, w+8 and B groups w, w+8 (4 DMAs per lane).
__device__ __forceinline__ void p9_issue(const LmHeadArgs& a, char* smem, int m0, int n0, int kt, int wave, int lane) {
    char* slot = smem + (kt & 3) * kP9Slot;
    const int rl = lane >> 2, pc = lane & 3;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int g = i * 8 + wave;
        const int r = g * 16 + rl;
        const uint16_t* src = a.h + int64_t(min(m0 + r, a.N - 1)) * a.ldh + kt * kP9BK + lds_chunk64(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(slot + g * 1024), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int g = i * 8 + wave;
        const int r = g * 16 + rl;
        const uint16_t* src = a.w + int64_t(min(n0 + r, a.V - 1)) * a.ldw + kt * kP9BK + lds_chunk64(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(slot + LmBig::BM * 64 + g * 1024),
                                         16, 0, 0);
    }
}

__global__ __launch_bounds__(512) void k_lmhead_pp9(LmHeadArgs a) {
    typedef LmBig G;
    __shared__ __attribute__((aligned(16))) char smem[kP9Lds];  // ONE LDS object (glds waits)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / G::WN, wc = wave % G::WN;
    const int ntt = (a.N + G::BM - 1) / G::BM;
    int b = blockIdx.x;
    if (a.xcd_swizzle) {
        const int nwg = gridDim.x, q = nwg / 8, r = nwg % 8, x = b % 8;
        b = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
    }
    const int mt = b % ntt, vt = b / ntt;
    const int m0 = mt * G::BM, n0 = vt * G::BN;
    float2* cmb = reinterpret_cast<float2*>(smem + 4 * kP9Slot);
    const int* lab = reinterpret_cast<const int*>(smem + kP9LabOff);
    // labels (low dwords) by LDS DMA first: an ordinary load would make hipcc drain the queue
    if (wave < 4) {
        const int64_t* src = a.labels + int64_t(min(m0 + wave * 64 + lane, a.N - 1)) * a.lb;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(smem + kP9LabOff + wave * 256),
                                         4, 0, 0);
    }
    f32x4_t acc[G::kMR][G::kNR];
#pragma unroll
    for (int i = 0; i < G::kMR; ++i)
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const int nk = a.H / kP9BK;  // even, >= 2
    p9_issue(a, smem, m0, n0, 0, wave, lane);
    p9_issue(a, smem, m0, n0, 1, wave, lane);
    if (nk > 2) {
        p9_issue(a, smem, m0, n0, 2, wave, lane);
        asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // labels + K-step 0 landed
    } else {
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    pp_barrier();
    if (wr == 1) pp_barrier();
    bf16x8_t af[8], bfr[4];
    const int fr = lane & 15, fc = lane >> 4;
    for (int kt = 0; kt < nk; ++kt) {
        const char* At = smem + (kt & 3) * kP9Slot;
        const char* Bt = At + G::BM * 64;
        if (!(a.dbg & 4)) {
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = lds_frag64(Bt, wc * 64 + j * 16 + fr, fc);
#pragma unroll
            for (int i = 0; i < 8; ++i) af[i] = lds_frag64(At, wr * 128 + i * 16 + fr, fc);
        }
        if (kt + 3 < nk) {
            if (!(a.dbg & 2)) p9_issue(a, smem, m0, n0, kt + 3, wave, lane);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // K-step kt+1 landed
        } else if (kt + 2 < nk) {
            asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // reads retired: the slot may be restaged
        pp_barrier();
        __builtin_amdgcn_s_setprio(1);
        if (!(a.dbg & 1)) {
#pragma unroll
            for (int i = 0; i < 8; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
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

// ------------------------------------------------------------------ persistent ping-pong
// k_lmhead_pingpong's schedule as ONE stream over all of a workgroup's tiles (tile j of
// workgroup b is b + j·gridDim): the half-tile stream, its slots (parity of the GLOBAL
// K-step count) and the counted waits run straight across tile boundaries, so a tile's
// first operands are already in LDS when its predecessor's last MFMAs retire.  Per tile:
//   * its labels (low dwords, 2 KB) arrive by LDS DMA issued just before the tile's first
//     half-tile, into a label buffer of the tile's parity (an ordinary load would make hipcc
//     drain the DMA queue; the extra DMA only makes later counted waits more conservative:
//     vector-memory ops retire in issue order);
//   * the epilogue is per wave group: the four waves of a wave row own the same 128 token
//     rows, so a group publishes its (max, Σexp) partials to LDS, passes ONE barrier and
//     merges them — group 0's epilogue runs beside group 1's last MFMA phase.
constexpr int kPPLabOff = kPPStageBytes + LmBig::WN * LmBig::BM * 8;  // int32 [2][256]
constexpr int kPPLabRing = 4;  // label buffers: tile j+4's DMA is issued after tile j's epilogue even at H = 64
constexpr int kPP2Lds = kPPLabOff + kPPLabRing * LmBig::BM * 4;

__device__ __forceinline__ void pp2_issue(const LmHeadArgs& a, char* smem, int m0, int n0, int kt, int kind,
                                          int parity, int wave, int lane) {
    char* slot = smem + (parity * 4 + kind) * kPPHalf;
    const int rl = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int g = i * 8 + wave;
        const int r = g * 8 + rl;
        const uint16_t* src;
        if (kind == 0 || kind == 3) {
            const int tr = (r >> 6) * 128 + (kind == 3 ? 64 : 0) + (r & 63);
            src = a.h + int64_t(min(m0 + tr, a.N - 1)) * a.ldh;
        } else {
            const int tc = (r >> 5) * 64 + (kind == 2 ? 32 : 0) + (r & 31);
            src = a.w + int64_t(min(n0 + tc, a.V - 1)) * a.ldw;
        }
        src += kt * kLmBK + lds_chunk(r, pc) * 8;
        __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(slot + g * 1024), 16, 0, 0);
    }
}

// Labels of the tile at m0 -> int32 lab[parity][256] (waves 0-3: 64 rows each).
__device__ __forceinline__ void pp2_issue_labels(const LmHeadArgs& a, char* smem, int m0, int parity, int wave,
                                                 int lane) {
    if (wave >= 4) return;
    const int r = wave * 64 + lane;
    const int64_t* src = a.labels + int64_t(min(m0 + r, a.N - 1)) * a.lb;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(smem + kPPLabOff +
                                                                                    parity * 1024 + wave * 256),
                                     4, 0, 0);
}

typedef int i32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ i32x4_t lds_load_i4(const int* p) {
    const uint32_t addr = uint32_t(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const int*)p));
    i32x4_t v;
    asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    return v;
}

__global__ __launch_bounds__(512) void k_lmhead_pp_persist(LmHeadArgs a, int ntiles) {
    typedef LmBig G;
    __shared__ __attribute__((aligned(16))) char smem[kPP2Lds];  // ONE LDS object (glds waits)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / G::WN, wc = wave % G::WN;
    const int ntt = (a.N + G::BM - 1) / G::BM;
    const int nk = a.H / kLmBK;
    const int mine = (ntiles - int(blockIdx.x) + int(gridDim.x) - 1) / int(gridDim.x);
    if (mine <= 0) return;
    const int SK = mine * nk;  // K-steps in this workgroup's stream
    const int S = 4 * SK;      // half-tiles (= phases)
    float2* cmb = reinterpret_cast<float2*>(smem + kPPStageBytes);
    const int* labs = reinterpret_cast<const int*>(smem + kPPLabOff);

    auto tile_origin = [&](int j, int& m0, int& n0) {
        const int t = int(blockIdx.x) + j * int(gridDim.x);
        m0 = (t % ntt) * G::BM;
        n0 = (t / ntt) * G::BN;
    };
    // Issue targets run 1-2 K-steps ahead of consumption, so they lie in the current tile or
    // the next one: both origins are kept as wave-uniform scalars (no per-issue division).
    int cm0, cn0, xm0, xn0;  // current tile j / next tile j+1
    tile_origin(0, cm0, cn0);
    tile_origin(1, xm0, xn0);
    // half-tile `kind` of K-step kt + d of tile j (d in {0, 1, 2}); g = global K-step index
    auto issue_at = [&](int j, int kt, int d, int kind, int g) __attribute__((always_inline)) {
        if (a.dbg & 2) return;
        int t_kt = kt + d, m0 = cm0, n0 = cn0, jj = j;
        if (t_kt >= nk) {
            t_kt -= nk;
            m0 = xm0;
            n0 = xn0;
            jj = j + 1;
            if (t_kt >= nk) {  // nk == 1: two K-steps ahead is tile j + 2
                t_kt -= nk;
                jj = j + 2;
                tile_origin(jj, m0, n0);
            }
        }
        if (t_kt == 0 && kind == 0) pp2_issue_labels(a, smem, m0, jj % kPPLabRing, wave, lane);
        pp2_issue(a, smem, m0, n0, t_kt, kind, (g + d) & 1, wave, lane);
    };

    f32x4_t acc[G::kMR][G::kNR];
#pragma unroll
    for (int i = 0; i < G::kMR; ++i)
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    for (int s2 = 0; s2 < 6; ++s2) issue_at(0, 0, s2 >> 2, s2 & 3, 0);  // K-steps 0 and 1 (1: maybe tile 1)
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // K-step 0's q0 operands (+ tile 0 labels) landed
    pp_barrier();
    if (wr == 1) pp_barrier();  // group 1 runs one barrier behind

    bf16x8_t af[2][4];
    bf16x8_t bfr[2][2][2];
    const int fr = lane & 15, fc = lane >> 4;

    auto phase = [&](int j, int kt, int g, auto qc, auto steadyc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        constexpr bool steady = decltype(steadyc)::value;
        const char* buf = smem + (g & 1) * 4 * kPPHalf;
        const int ph = 4 * g + q;
        // issue target: half-tile ph + 6 = K-step g + 1 (kinds 2, 3) or g + 2 (kinds 0, 1)
        constexpr int d = q < 2 ? 1 : 2;
        constexpr int kind = (q + 2) & 3;
        if constexpr (q == 0 || q == 2) {
            if (!(a.dbg & 4)) {
            const char* At = buf + (q == 0 ? 0 : 3) * kPPHalf;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < 4; ++i) af[ks][i] = lds_frag(At, wr * 64 + i * 16 + fr, ks * 4 + fc);
            }
        }
        if constexpr (q == 0 || q == 1) {
            if (!(a.dbg & 4)) {
            const char* Bt = buf + (q == 0 ? 1 : 2) * kPPHalf;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int j = 0; j < 2; ++j) bfr[q][ks][j] = lds_frag(Bt, wc * 32 + j * 16 + fr, ks * 4 + fc);
            }
        }
        if constexpr (steady) {
            issue_at(j, kt, d, kind, g);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
        } else {
            if (ph + 6 < S) issue_at(j, kt, d, kind, g);
            const int n = min(ph + 6, S - 1) - (ph + 2);
            pp_wait(n < 0 ? 0 : (n > 4 ? 4 : n));
        }
        pp_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        constexpr int qm = q >= 2 ? 1 : 0;
        constexpr int qn = (q == 1 || q == 2) ? 1 : 0;
        __builtin_amdgcn_s_setprio(1);
        if (!(a.dbg & 1))
#pragma unroll
        for (int ks = 0; ks < 2; ++ks)
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[qm * 4 + i][qn * 2 + j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                        af[ks][i], bfr[qn][ks][j], acc[qm * 4 + i][qn * 2 + j], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
    };

    typedef std::integral_constant<bool, true> Steady;
    for (int j = 0; j < mine; ++j) {
        for (int kt = 0; kt < nk; ++kt) {
            const int g = j * nk + kt;
            // every phase is "steady": past the end of the stream the issues fetch clamped,
            // never-read rows of a phantom tile, so vmcnt(8) is exact throughout
            phase(j, kt, g, std::integral_constant<int, 0>{}, Steady{});
            phase(j, kt, g, std::integral_constant<int, 1>{}, Steady{});
            phase(j, kt, g, std::integral_constant<int, 2>{}, Steady{});
            phase(j, kt, g, std::integral_constant<int, 3>{}, Steady{});
        }
        // ---- tile epilogue, per wave group (see above).  acc[I][J][r] at lane l =
        // logit(token m0 + wr*128 + I*16 + (l>>4)*4 + r, vocab n0 + wc*64 + J*16 + (l&15))
        const int m0 = cm0, n0 = cn0;
        const int vt = n0 / G::BN;
        const int* lab = labs + (j % kPPLabRing) * G::BM;
        // lane-derived bases laundered here: otherwise hipcc hoists the 32 row addresses out
        // of the tile loop and spills them, and the scratch reloads wait vmcnt(0) (draining
        // the operand stream at every tile boundary)
        const int cl = launder_int(lane & 15);
        const int rbase = launder_int(wr * G::kWRows + (lane >> 4) * 4);
        float2* cmbw = cmb + launder_int(wc * G::BM);
#pragma unroll
        for (int i = 0; i < G::kMR; ++i) {
            const i32x4_t lab4 = lds_load_i4(lab + rbase + i * 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rt = rbase + i * 16 + q;
                float x[G::kNR];
                float mx = -INFINITY;
#pragma unroll
                for (int jj = 0; jj < G::kNR; ++jj) {
                    const int v = n0 + wc * G::kWCols + jj * 16 + cl;
                    x[jj] = v < a.V ? acc[i][jj][q] : -INFINITY;
                    mx = fmaxf(mx, x[jj]);
                }
                mx = row16_max(mx);
                const float ml2e = mx == -INFINITY ? 0.f : -mx * kLog2e;
                float sm = 0.f;
#pragma unroll
                for (int jj = 0; jj < G::kNR; ++jj) sm += exp2_fast(fmaf(x[jj], kLog2e, ml2e));
                sm = row16_sum(sm);
                if (cl == 0) lds_store_f2(cmbw + rt, mx, sm);
                const int dy = lab4[q] - (n0 + wc * G::kWCols);
                if (dy >= 0 && dy < G::kWCols && (dy & 15) == cl && m0 + rt < a.N) {
                    float xy = x[0];
#pragma unroll
                    for (int jj = 1; jj < G::kNR; ++jj) xy = (dy >> 4) == jj ? x[jj] : xy;
                    a.xlab[m0 + rt] = xy;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < G::kMR; ++i)
#pragma unroll
            for (int jj = 0; jj < G::kNR; ++jj) acc[i][jj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();  // the group's four waves published their partials
        {
            const int gt = tid - wr * 256;  // 0..255 within the group; rows wr*128 + [0, 128)
            if (gt < 128 && m0 + wr * 128 + gt < a.N) {
                const int r = wr * 128 + gt;
                float2 pw[G::WN];
                float m = -INFINITY;
#pragma unroll
                for (int c2 = 0; c2 < G::WN; ++c2) {
                    pw[c2] = lds_load_f2(cmb + c2 * G::BM + r);
                    m = fmaxf(m, pw[c2].x);
                }
                float sm = 0.f;
                if (m != -INFINITY) {
#pragma unroll
                    for (int c2 = 0; c2 < G::WN; ++c2)
                        sm += pw[c2].x == -INFINITY ? 0.f : pw[c2].y * exp2_fast((pw[c2].x - m) * kLog2e);
                }
                a.part[int64_t(m0 + r) * a.nvt + vt] = make_float2(m, sm);
            }
        }
        cm0 = xm0;
        cn0 = xn0;
        tile_origin(j + 2, xm0, xn0);
    }
    if (wr == 0) pp_barrier();  // balance group 1's extra barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------ persistent 2-phase ping-pong
// k_lmhead_pp2's schedule (2 phases of 32 MFMAs per 64-deep K-step) as ONE stream over all of
// a workgroup's tiles, as k_lmhead_pp_persist does for the 4-phase form: the half-tile stream
// (HA0/HB0/HB1 of K-step g+1 issued in phase A of step g, HA1(g+1) in phase B), its slots
// (parity of the global K-step index) and the counted waits (vmcnt(6) / vmcnt(2)) run across
// tile boundaries; labels arrive by LDS DMA just ahead of each tile's first half-tile; the
// epilogue is per wave group (one extra barrier per tile); past the end the issues fetch
// clamped rows of a phantom tile so the counts stay exact.
__global__ __launch_bounds__(512) void k_lmhead_pp2_persist(LmHeadArgs a, int ntiles) {
    typedef LmBig G;
    __shared__ __attribute__((aligned(16))) char smem[kPP2Lds];  // ONE LDS object (glds waits)
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave / G::WN, wc = wave % G::WN;
    const int ntt = (a.N + G::BM - 1) / G::BM;
    const int nk = a.H / kLmBK;
    const int mine = (ntiles - int(blockIdx.x) + int(gridDim.x) - 1) / int(gridDim.x);
    if (mine <= 0) return;
    float2* cmb = reinterpret_cast<float2*>(smem + kPPStageBytes);
    const int* labs = reinterpret_cast<const int*>(smem + kPPLabOff);
    auto tile_origin = [&](int j, int& m0, int& n0) {
        const int t = int(blockIdx.x) + j * int(gridDim.x);
        m0 = (t % ntt) * G::BM;
        n0 = (t / ntt) * G::BN;
    };
    int cm0, cn0, xm0, xn0;  // tile j / tile j+1 origins
    tile_origin(0, cm0, cn0);
    tile_origin(1, xm0, xn0);
    // kinds [k0, k1) of K-step kt+1 of tile j (global index g+1): the current tile or the next
    auto issue_next = [&](int j, int kt, int g, int k0, int k1) __attribute__((always_inline)) {
        int t_kt = kt + 1, m0 = cm0, n0 = cn0, jj = j;
        if (t_kt >= nk) {
            t_kt = 0;
            m0 = xm0;
            n0 = xn0;
            jj = j + 1;
        }
        (void)jj;
        for (int kind = k0; kind < k1; ++kind) pp2_issue(a, smem, m0, n0, t_kt, kind, (g + 1) & 1, wave, lane);
    };

    f32x4_t acc[G::kMR][G::kNR];
#pragma unroll
    for (int i = 0; i < G::kMR; ++i)
#pragma unroll
        for (int j = 0; j < G::kNR; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    // prologue: tile 0's labels and all of K-step 0; HA0/HB0/HB1 retired, HA1 may stay in flight
    pp2_issue_labels(a, smem, cm0, 0, wave, lane);
#pragma unroll
    for (int kind = 0; kind < 4; ++kind) pp2_issue(a, smem, cm0, cn0, 0, kind, 0, wave, lane);
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    pp_barrier();
    if (wr == 1) pp_barrier();  // group 1 runs one barrier behind
    bf16x8_t af[2][4];
    bf16x8_t bfr[2][2][2];
    const int fr = lane & 15, fc = lane >> 4;
    for (int j = 0; j < mine; ++j) {
        for (int kt = 0; kt < nk; ++kt) {
            const int g = j * nk + kt;
            const char* buf = smem + (g & 1) * 4 * kPPHalf;
            // ---- phase A: rows qm = 0
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < 4; ++i) af[ks][i] = lds_frag(buf, wr * 64 + i * 16 + fr, ks * 4 + fc);
#pragma unroll
            for (int qn = 0; qn < 2; ++qn)
#pragma unroll
                for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                    for (int jj = 0; jj < 2; ++jj)
                        bfr[qn][ks][jj] = lds_frag(buf + (1 + qn) * kPPHalf, wc * 32 + jj * 16 + fr, ks * 4 + fc);
            issue_next(j, kt, g, 0, 3);
            if (kt == 0 && wave < 4) {  // tile j+1's labels, youngest op: counted exactly
                pp2_issue_labels(a, smem, xm0, (j + 1) % kPPLabRing, wave, lane);
                asm volatile("s_waitcnt vmcnt(7)" ::: "memory");  // HA1(g) landed
            } else {
                asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // HA1(g) landed
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
                        for (int jj = 0; jj < 2; ++jj)
                            acc[i][qn * 2 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                af[ks][i], bfr[qn][ks][jj], acc[i][qn * 2 + jj], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            pp_barrier();
            // ---- phase B: rows qm = 1
#pragma unroll
            for (int ks = 0; ks < 2; ++ks)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    af[ks][i] = lds_frag(buf + 3 * kPPHalf, wr * 64 + i * 16 + fr, ks * 4 + fc);
            issue_next(j, kt, g, 3, 4);
            asm volatile("s_waitcnt vmcnt(2)" ::: "memory");  // K-step g+1's HA0/HB0/HB1 landed
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
                        for (int jj = 0; jj < 2; ++jj)
                            acc[4 + i][qn * 2 + jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                af[ks][i], bfr[qn][ks][jj], acc[4 + i][qn * 2 + jj], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
            pp_barrier();
        }
        // ---- tile epilogue, per wave group (k_lmhead_pp_persist's)
        const int m0 = cm0, n0 = cn0;
        const int vt = n0 / G::BN;
        const int* lab = labs + (j % kPPLabRing) * G::BM;
        const int cl = launder_int(lane & 15);
        const int rbase = launder_int(wr * G::kWRows + (lane >> 4) * 4);
        float2* cmbw = cmb + launder_int(wc * G::BM);
#pragma unroll
        for (int i = 0; i < G::kMR; ++i) {
            const i32x4_t lab4 = lds_load_i4(lab + rbase + i * 16);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int rt = rbase + i * 16 + q;
                float x[G::kNR];
                float mx = -INFINITY;
#pragma unroll
                for (int jj = 0; jj < G::kNR; ++jj) {
                    const int v = n0 + wc * G::kWCols + jj * 16 + cl;
                    x[jj] = v < a.V ? acc[i][jj][q] : -INFINITY;
                    mx = fmaxf(mx, x[jj]);
                }
                mx = row16_max(mx);
                const float ml2e = mx == -INFINITY ? 0.f : -mx * kLog2e;
                float sm = 0.f;
#pragma unroll
                for (int jj = 0; jj < G::kNR; ++jj) sm += exp2_fast(fmaf(x[jj], kLog2e, ml2e));
                sm = row16_sum(sm);
                if (cl == 0) lds_store_f2(cmbw + rt, mx, sm);
                const int dy = lab4[q] - (n0 + wc * G::kWCols);
                if (dy >= 0 && dy < G::kWCols && (dy & 15) == cl && m0 + rt < a.N) {
                    float xy = x[0];
#pragma unroll
                    for (int jj = 1; jj < G::kNR; ++jj) xy = (dy >> 4) == jj ? x[jj] : xy;
                    a.xlab[m0 + rt] = xy;
                }
            }
        }
#pragma unroll
        for (int i = 0; i < G::kMR; ++i)
#pragma unroll
            for (int jj = 0; jj < G::kNR; ++jj) acc[i][jj] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        pp_barrier();  // the group's four waves published their partials
        {
            const int gt = tid - wr * 256;
            if (gt < 128 && m0 + wr * 128 + gt < a.N) {
                const int r = wr * 128 + gt;
                float2 pw[G::WN];
                float m = -INFINITY;
#pragma unroll
                for (int c2 = 0; c2 < G::WN; ++c2) {
                    pw[c2] = lds_load_f2(cmb + c2 * G::BM + r);
                    m = fmaxf(m, pw[c2].x);
                }
                float sm = 0.f;
                if (m != -INFINITY) {
#pragma unroll
                    for (int c2 = 0; c2 < G::WN; ++c2)
                        sm += pw[c2].x == -INFINITY ? 0.f : pw[c2].y * exp2_fast((pw[c2].x - m) * kLog2e);
                }
                a.part[int64_t(m0 + r) * a.nvt + vt] = make_float2(m, sm);
            }
        }
        cm0 = xm0;
        cn0 = xn0;
        tile_origin(j + 2, xm0, xn0);
    }
    if (wr == 0) pp_barrier();  // balance group 1's extra barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// One wave per token: merge the nvt partials (fixed order per lane, then a fixed butterfly).
__global__ __launch_bounds__(256) void k_lmhead_combine(LmHeadArgs a, void* lp, int lp_dtype, float* lse_out) {
    const int lane = threadIdx.x & 63;
    const int64_t n = int64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (n >= a.N) return;
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
    // label logit: picked out by the tile kernel (xlab), or recomputed here as h[n]·W[y]
    // (fp32 sum of the same exact bf16 products; one H-long dot per token)
    const int64_t y = a.labels[n * a.lb];
    const bool y_ok = y >= 0 && y < a.V;
    float xy = 0.f;
    if (a.xlab == nullptr && y_ok) {
        const uint32_t* hr = reinterpret_cast<const uint32_t*>(a.h + n * a.ldh);
        const uint32_t* wr = reinterpret_cast<const uint32_t*>(a.w + y * a.ldw);
        for (int k = lane; k < a.H / 2; k += kWave) {
            const uint32_t hv = hr[k], wv = wr[k];
            xy = fmaf(bf_lo(hv), bf_lo(wv), xy);
            xy = fmaf(bf_hi(hv), bf_hi(wv), xy);
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) xy += __shfl_xor(xy, off, kWave);
    }
    if (lane == 0) {
        const float lse = m + logf(s);
        if (a.xlab) xy = a.xlab[n];
        const float lpv = y_ok ? xy - lse : NAN;
        st_any(lp, lp_dtype, n, lpv);
        if (lse_out) lse_out[n] = lse;
    }
}

}  // namespace trlx

using namespace trlx;

// variant: 0 auto, 1 persistent 256x256 (BK 32, 3 stages in flight), 2 256x256 tiles, 3 128x128
// tiles, 4 = 2 with the XCD remap, 5 ping-pong 4 phases per K-step, 6 = 5 with the XCD remap,
// 7 persistent ping-pong, 8 ping-pong 2 phases per K-step.
// auto (measured on MI355X, tools/lmhead_bench.py, interleaved rounds): N >= 2048 -> 8 (the
// fastest at every BASELINE shape: 1.1-1.4x the 2-barrier tiles); small N -> 128x128 tiles
// (enough workgroups to fill 256 CUs).
static int g_lm_variant = 0;
static int g_lm_dbg = 0;  // ping-pong ablation bits, set via trlx_set_tuning("lmhead_dbg") (timing probes)
static int lm_variant(int64_t N, int64_t H = 0) {
    (void)H;
    if (g_lm_variant) return g_lm_variant;
    return N < 2048 ? 3 : 8;
}
static int lm_tile_n(int64_t N) { return lm_variant(N) == 3 ? LmSmall::BN : LmBig::BN; }
static_assert(LmSmall::BN == 128 && LmBig::BN == 256, "tile widths");

namespace trlx {
void lm_set_dbg(int v) { g_lm_dbg = v; }
}  // namespace trlx

extern "C" int trlx_lmhead_set_variant(int v) {
    TRLX_REQUIRE(v >= 0 && v <= 10, TRLX_ERR_ARG, "lmhead variant 0..10");
    g_lm_variant = v;
    return TRLX_OK;
}

static int lm_num_cus() {
    static int n = 0;
    if (n == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template <class G>
static int lm_launch_persist(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntiles = int64_t((a.N + G::BM - 1) / G::BM) * a.nvt;
    TRLX_REQUIRE(ntiles < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    const int grid = int(ntiles < lm_num_cus() ? ntiles : lm_num_cus());
    LmHeadArgs b = a;
    b.xlab = nullptr;  // the combine kernel recomputes the label logit
    hipLaunchKernelGGL((k_lmhead_persist<G>), dim3(grid), dim3(G::kThreads), 0, stream, b, int(ntiles));
    return check_launch("k_lmhead_persist");
}

extern "C" int64_t trlx_lmhead_workspace_bytes(int64_t N, int64_t V) {
    const int64_t nvt = (V + lm_tile_n(N) - 1) / lm_tile_n(N);
    return N * nvt * int64_t(sizeof(float2)) + N * int64_t(sizeof(float));
}

template <class G>
static int lm_launch(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntt = (a.N + G::BM - 1) / G::BM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    hipLaunchKernelGGL((k_lmhead_tiles<G>), dim3(unsigned(ntt * a.nvt)), dim3(G::kThreads), 0, stream, a);
    return check_launch("k_lmhead_tiles");
}

static int lm_launch_pp_persist(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntiles = int64_t((a.N + LmBig::BM - 1) / LmBig::BM) * a.nvt;
    TRLX_REQUIRE(ntiles < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    const int grid = int(ntiles < lm_num_cus() ? ntiles : lm_num_cus());
    hipLaunchKernelGGL(k_lmhead_pp_persist, dim3(grid), dim3(512), 0, stream, a, int(ntiles));
    return check_launch("k_lmhead_pp_persist");
}

static int lm_launch_pp2(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntt = (a.N + LmBig::BM - 1) / LmBig::BM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    hipLaunchKernelGGL(k_lmhead_pp2, dim3(unsigned(ntt * a.nvt)), dim3(512), 0, stream, a);
    return check_launch("k_lmhead_pp2");
}

static int lm_launch_pp2_persist(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntiles = int64_t((a.N + LmBig::BM - 1) / LmBig::BM) * a.nvt;
    TRLX_REQUIRE(ntiles < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    const int grid = int(ntiles < lm_num_cus() ? ntiles : lm_num_cus());
    hipLaunchKernelGGL(k_lmhead_pp2_persist, dim3(grid), dim3(512), 0, stream, a, int(ntiles));
    return check_launch("k_lmhead_pp2_persist");
}

static int lm_launch_pp9(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntt = (a.N + LmBig::BM - 1) / LmBig::BM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    hipLaunchKernelGGL(k_lmhead_pp9, dim3(unsigned(ntt * a.nvt)), dim3(512), 0, stream, a);
    return check_launch("k_lmhead_pp9");
}

static int lm_launch_pingpong(const LmHeadArgs& a, hipStream_t stream) {
    const int64_t ntt = (a.N + LmBig::BM - 1) / LmBig::BM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    hipLaunchKernelGGL(k_lmhead_pingpong, dim3(unsigned(ntt * a.nvt)), dim3(512), 0, stream, a);
    return check_launch("k_lmhead_pingpong");
}

extern "C" int trlx_lmhead_logprobs(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                    int64_t H, int64_t V, const int64_t* labels, int64_t lb, void* lp_out,
                                    int lp_dtype, float* lse_out, void* workspace, void* stream) {
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
    const int bn = lm_tile_n(N);
    a.nvt = int((V + bn - 1) / bn);
    a.part = static_cast<float2*>(workspace);
    a.xlab = reinterpret_cast<float*>(static_cast<char*>(workspace) + N * a.nvt * int64_t(sizeof(float2)));
    const int var = lm_variant(N, H);
    a.xcd_swizzle = var == 4 || var == 6;
    a.dbg = g_lm_dbg;
    int rc = var == 10             ? lm_launch_pp2_persist(a, (hipStream_t)stream)
             : var == 9            ? lm_launch_pp9(a, (hipStream_t)stream)
             : var == 8            ? lm_launch_pp2(a, (hipStream_t)stream)
             : var == 7            ? lm_launch_pp_persist(a, (hipStream_t)stream)
             : var == 5 || var == 6 ? lm_launch_pingpong(a, (hipStream_t)stream)
             : var == 1            ? lm_launch_persist<LmBig>(a, (hipStream_t)stream)
             : var == 2 || var == 4 ? lm_launch<LmBig>(a, (hipStream_t)stream)
                                    : lm_launch<LmSmall>(a, (hipStream_t)stream);
    if (rc) return rc;
    LmHeadArgs c = a;
    if (var == 1) c.xlab = nullptr;
    hipLaunchKernelGGL(k_lmhead_combine, dim3(unsigned((N + 3) / 4)), dim3(256), 0, (hipStream_t)stream, c, lp_out,
                       lp_dtype, lse_out);
    return check_launch("k_lmhead_combine");
}
