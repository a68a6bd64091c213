// Fused lm_head projection + log-softmax-gather: logprobs of the labels
// straight from the decoder's hidden states, the [N, V] logits never written to HBM.
//
//   lp[n] = h[n]·W[y_n] − logsumexp_v(h[n]·W[v])        h [N, H] bf16, W [V, H] bf16 (nn.Linear)
//
// Replaces `logits = lm_head(hs)` (T5HeadWithValueModel, ppo_models.py:640; GPT lm_head :274,
// :588) followed by logprobs_from_logits (modeling.py:37-41) on the experience side
// (ppo_orchestrator.py:135-155), where no gradient is needed.  Two launches:
//
//   k_lmhead_tiles    MFMA GEMM over 128 tokens x 128 vocab tiles (K = H streamed in 64-deep
//                     steps through double-buffered LDS by global_load_lds, 16 B per lane, an
//                     XOR-swizzled image read conflict-free with ds_read_b128); the epilogue
//                     reduces each token's 128 logits of the tile to a partial (max, Σexp)
//                     and the tile that holds the label stores its logit.
//   k_lmhead_combine  one wave per token merges its V/128 partials -> lse, lp = x_y − lse.
//
// The GEMM is MFMA-bound (2·H FLOP per token·vocab pair); the partials cost 8 B per
// (token, vocab tile) — 1/16 of writing the bf16 logits.
#include "common.h"

namespace trlx {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int kLmBM = 128;               // tokens per tile
constexpr int kLmBN = 128;               // vocab entries per tile
constexpr int kLmBK = 64;                // K per stage (one 128-B row of bf16 per tile row)
constexpr int kLmThreads = 256;          // 4 waves, 2 (tokens) x 2 (vocab), 64 x 64 each
constexpr int kLmStage = (kLmBM + kLmBN) * kLmBK * 2;  // 32 KB: A tile + B tile
constexpr int kLmLds = 2 * kLmStage + kLmBM * 4;       // double buffer + the tile's labels

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
};

// Swizzled LDS image of a [128 rows][64 k] bf16 tile: row r is 128 B; its 16-B chunk c sits
// at physical chunk c ^ ((r >> 1) & 7).  A quarter-wave ds_read_b128 of one chunk column
// over 16 consecutive rows then touches 16 distinct 4-bank groups (even / odd rows fall in
// the two halves of the 256-B bank row): conflict-free.
__device__ __forceinline__ int lds_chunk(int r, int c) { return c ^ ((r >> 1) & 7); }

// Stage k-step `kt` of the A (tokens) and B (vocab) tiles into `stage`: 16 wave-instructions
// of 1 KB (8 rows) per operand, 4 + 4 per wave; each lane fetches the logical chunk that
// lands at its lane-linear LDS slot.  Rows past N / V are clamped (their results are masked).
__device__ __forceinline__ void lm_stage(const LmHeadArgs& a, char* stage, int m0, int n0, int kt, int wave,
                                         int lane) {
    const int rl = lane >> 3, pc = lane & 7;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int g = wave * 4 + i;   // 8-row group
        const int r = g * 8 + rl;
        const int lc = lds_chunk(r, pc);  // the involution maps physical -> logical too
        const int ma = min(m0 + r, a.N - 1);
        const uint16_t* srcA = a.h + int64_t(ma) * a.ldh + kt * kLmBK + lc * 8;
        __builtin_amdgcn_global_load_lds(srcA, (__attribute__((address_space(3))) void*)(stage + g * 1024), 16, 0,
                                         0);
        const int nb = min(n0 + r, a.V - 1);
        const uint16_t* srcB = a.w + int64_t(nb) * a.ldw + kt * kLmBK + lc * 8;
        __builtin_amdgcn_global_load_lds(srcB, (__attribute__((address_space(3))) void*)(stage + kLmBM * 128 + g * 1024),
                                         16, 0, 0);
    }
}

__device__ __forceinline__ bf16x8_t lds_frag(const char* tile, int r, int c) {
    return *reinterpret_cast<const bf16x8_t*>(tile + r * 128 + lds_chunk(r, c) * 16);
}

__global__ __launch_bounds__(kLmThreads) void k_lmhead_tiles(LmHeadArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[kLmLds];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wr = wave >> 1, wc = wave & 1;
    // token tiles fastest: consecutive workgroups share the vocab tile (its W rows stay in L2)
    const int ntt = (a.N + kLmBM - 1) / kLmBM;
    const int mt = blockIdx.x % ntt, vt = blockIdx.x / ntt;
    const int m0 = mt * kLmBM, n0 = vt * kLmBN;
    int* lab = reinterpret_cast<int*>(smem + 2 * kLmStage);
    if (tid < kLmBM) {
        const int m = m0 + tid;
        lab[tid] = m < a.N ? int(a.labels[int64_t(m) * a.lb]) : -1;
    }

    f32x4_t acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

    const int nk = a.H / kLmBK;
    lm_stage(a, smem, m0, n0, 0, wave, lane);
    for (int kt = 0; kt < nk; ++kt) {
        char* cur = smem + (kt & 1) * kLmStage;
        if (kt + 1 < nk) {
            lm_stage(a, smem + ((kt + 1) & 1) * kLmStage, m0, n0, kt + 1, wave, lane);
            asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // tile kt landed, kt+1 in flight
        } else {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_s_barrier();
        const char* At = cur;
        const char* Bt = cur + kLmBM * 128;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            const int c = ks * 4 + (lane >> 4);
            bf16x8_t af[4], bfr[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) af[i] = lds_frag(At, wr * 64 + i * 16 + (lane & 15), c);
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[j] = lds_frag(Bt, wc * 64 + j * 16 + (lane & 15), c);
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        }
        __builtin_amdgcn_s_barrier();  // every wave is done reading `cur` before it is restaged
    }

    // ---- epilogue: per token row, the tile's partial (max, Σexp) and the label logit
    // acc[i][j][q] at lane l = logit(token m0 + wr*64 + i*16 + (l>>4)*4 + q,
    //                                 vocab n0 + wc*64 + j*16 + (l&15))
    float2* cmb = reinterpret_cast<float2*>(smem);  // [2 wc][128 rows], staging is free now
    const int cl = lane & 15;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int rt = wr * 64 + i * 16 + (lane >> 4) * 4 + q;  // row in tile
            float x[4];
            float mx = -INFINITY;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int v = n0 + wc * 64 + j * 16 + cl;
                x[j] = v < a.V ? acc[i][j][q] : -INFINITY;
                mx = fmaxf(mx, x[j]);
            }
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, kWave));
            // a fully masked row piece (columns >= V) keeps (-inf, 0): exp(-inf - -inf) is NaN
            const float ml2e = mx == -INFINITY ? 0.f : -mx * kLog2e;
            float s = 0.f;
#pragma unroll
            for (int j = 0; j < 4; ++j) s += exp2_fast(fmaf(x[j], kLog2e, ml2e));
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) s += __shfl_xor(s, off, kWave);
            if (cl == 0) cmb[wc * kLmBM + rt] = make_float2(mx, s);
            const int dy = lab[rt] - (n0 + wc * 64);
            if (dy >= 0 && dy < 64 && (dy & 15) == cl && m0 + rt < a.N) {
                const int jy = dy >> 4;
                a.xlab[m0 + rt] = jy == 0 ? x[0] : jy == 1 ? x[1] : jy == 2 ? x[2] : x[3];
            }
        }
    }
    __syncthreads();
    if (tid < kLmBM && m0 + tid < a.N) {
        const float2 p0 = cmb[tid], p1 = cmb[kLmBM + tid];
        const float m = fmaxf(p0.x, p1.x);
        float s = 0.f;
        if (m != -INFINITY)
            s = (p0.x == -INFINITY ? 0.f : p0.y * exp2_fast((p0.x - m) * kLog2e)) +
                (p1.x == -INFINITY ? 0.f : p1.y * exp2_fast((p1.x - m) * kLog2e));
        a.part[int64_t(m0 + tid) * a.nvt + vt] = make_float2(m, s);
    }
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
    if (lane == 0) {
        const float lse = m + logf(s);
        const int64_t y = a.labels[n * a.lb];
        const float lpv = (y >= 0 && y < a.V) ? a.xlab[n] - lse : NAN;
        st_any(lp, lp_dtype, n, lpv);
        if (lse_out) lse_out[n] = lse;
    }
}

}  // namespace trlx

using namespace trlx;

extern "C" int64_t trlx_lmhead_workspace_bytes(int64_t N, int64_t V) {
    const int64_t nvt = (V + kLmBN - 1) / kLmBN;
    return N * nvt * int64_t(sizeof(float2)) + N * int64_t(sizeof(float));
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
    a.nvt = int((V + kLmBN - 1) / kLmBN);
    a.part = static_cast<float2*>(workspace);
    a.xlab = reinterpret_cast<float*>(static_cast<char*>(workspace) + N * a.nvt * int64_t(sizeof(float2)));
    const int64_t ntt = (N + kLmBM - 1) / kLmBM;
    TRLX_REQUIRE(ntt * a.nvt < (int64_t(1) << 31), TRLX_ERR_SHAPE, "too many tiles");
    hipLaunchKernelGGL(k_lmhead_tiles, dim3(unsigned(ntt * a.nvt)), dim3(kLmThreads), 0, (hipStream_t)stream, a);
    int rc = check_launch("k_lmhead_tiles");
    if (rc) return rc;
    hipLaunchKernelGGL(k_lmhead_combine, dim3(unsigned((N + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a, lp_out,
                       lp_dtype, lse_out);
    return check_launch("k_lmhead_combine");
}
