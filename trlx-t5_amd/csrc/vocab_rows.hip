// Vocab-axis row kernels: fused log-softmax + gather (forward), its backward, and the
// loss-side fused forward+backward (logprob -> PPO policy gradient -> dlogits); the fused
// step's rollout-level [T]-vector work runs in one-wave-per-rollout kernels (row_tails.h).
//
// One workgroup owns one logits row (b, t) of V elements.  Register-resident variant: the
// row is loaded ONCE from HBM into VGPRs as 16-byte buffer loads (NV per thread, all in
// flight up front), max and sum-exp are wavefront-shuffle + LDS block reductions, and the
// backward / fused kernels write dlogits from the same registers: 1 read (+1 write) of
// V*s bytes per token, never materialising the [B,T,V] log-softmax the reference builds
// (trlx/utils/modeling.py:39).  Streaming variant: online (max, sum-exp) over U vectors
// in flight per thread, for rows too long to hold.  No MFMA: nothing here is a
// contraction; the roofline is HBM bandwidth.
#include <string>

#include <hip/hip_ext.h>

#include "ppo_token.h"
#include "row_order.h"

namespace trlx {

enum RowMode { kFwd = 0, kBwd = 1, kPpo = 2 };

struct RowArgs {
    const void* x0;           // logits (tensor 0)
    const void* x1;           // second logits tensor (fwd only; blockIdx.y == 1)
    int64_t B, T, V, sb, st;  // shape + token strides (elements)
    const int64_t* labels;
    int64_t lb, lt;
    // forward outputs
    void* lp0;
    void* lp1;
    int out_dtype;
    float* lse0;
    float* lse1;
    // backward inputs
    const float* lse_in;
    const void* grad;
    int grad_dtype;
    // ppo fused inputs
    const void* old_lp;
    int old_dtype;
    const float* adv;
    const double* stats;
    int unbiased;
    int order;                // vector order of the resident rows (0 step-major, 1 wave-major)
    int spol;                 // gradient-row store cache policy (tuning "store_policy", see g_store_pol)
    const int64_t* mask;
    const double* msum;
    double msum_host;
    float cliprange;
    float* lp_out;
    // gradient output (bwd / ppo)
    void* dx;
    int64_t dsb, dst;
    // fused loss: per-token loss records + value gradient (row_tails.h)
    float* tokrec;
    LossTokenArgs ltok;
    // forward only: the PREVIOUS step's loss tail folded into this launch as its first
    // `tail_blocks` workgroups (trlx_lsm_gather_fwd_loss_tail); row = blockIdx.x - tail_blocks
    int has_tail, tail_blocks;
    LossRolloutArgs tail;
    // loss rows only: the NEXT batch's split GAE folded into this launch as its first
    // `gae_blocks` workgroups (trlx_ppo_loss_rows_split_gae; no data dependency between them)
    int has_gae, gae_blocks;
    GaeRolloutArgs gae;
    int lead_blocks;          // tail_blocks + gae_blocks: row = blockIdx.x - lead_blocks
    void* done_event;         // host only: recorded by the launch's own dispatch (or NULL)
    // split-beta loss rows (trlx_ppo_loss_rows_split): adv = A0, A = A0 - beta*Ak whitened with
    // coef {mu, rstd, beta}; this launch also finishes the batch's rewards and returns
    const float* coef;
    const float* adv_kl;
    const float* rew_kl;
    const float* rew_score;
    float* rewards_out;
    // split-beta rows that derive the batch's whitening coefficients themselves (no coef
    // launch): whiten_coef_split(wstats, wunbiased, beta = wctl[KL_COEF] or wbeta), row 0
    // storing them to coef_out for later launches on the same experience (ppo_epochs)
    const double* wstats;
    int wunbiased;
    const double* wctl;
    float wbeta;
    float* coef_out;
    // forward rows of a ragged batch: rows (b, t >= lengths[b]) are store padding (pad_row)
    const int64_t* lengths;
    // ... and their dispatch order (k_ragged_order): workgroup i takes row row_list[i] (>= 0), or
    // writes the padding row ~row_list[i]; NULL: workgroup i takes row i
    const int* row_list;
    int* order_ws;            // host: int32 [B·T] scratch for the order (NULL: natural order)
};

// ------------------------------------------------------------------ shared row pieces
template <class DT>
struct Row {
    typedef typename DT::elem_t E;
    int64_t row, b, t;
    const E* x;
    int64_t y;
    bool y_ok;
    RowSplit<DT> s;
    __device__ __forceinline__ Row(const RowArgs& a) : Row(a, int64_t(blockIdx.x) - a.lead_blocks) {}
    __device__ __forceinline__ Row(const RowArgs& a, int64_t row_)
        : row(row_),
          b(row / a.T),
          t(row - b * a.T),
          x(reinterpret_cast<const E*>(blockIdx.y == 0 ? a.x0 : a.x1) + b * a.sb + t * a.st),
          y(a.labels[b * a.lb + t * a.lt]),
          y_ok(y >= 0 && y < a.V),
          s(x, a.V) {}
    // head element -> threads [0, head); tail element -> the last `tail` threads
    __device__ __forceinline__ int64_t edge_index() const {
        const int tid = threadIdx.x, nthr = blockDim.x;
        if (tid < s.head) return tid;
        if (tid >= nthr - s.tail) return s.tail0 + (tid - (nthr - s.tail));
        return -1;
    }
};

// Forward epilogue: write lp (+lse).
template <class DT>
__device__ __forceinline__ void fwd_epilogue(const RowArgs& a, const Row<DT>& r, float lp, float lse) {
    if (threadIdx.x == 0) {  // lp = (x[y] - max) - log Σ (NaN for an out-of-range label)
        st_any(blockIdx.y == 0 ? a.lp0 : a.lp1, a.out_dtype, r.row, lp);
        float* lse_out = blockIdx.y == 0 ? a.lse0 : a.lse1;
        if (lse_out) lse_out[r.row] = lse;
    }
}

// Per-token gradient scale g = d loss / d lp.
template <int MODE>
__device__ __forceinline__ float row_grad(const RowArgs& a, int64_t row, float lp, const PpoScalars& ps,
                                          PolicyTerms& pt) {
    if (MODE == kBwd) return ld_any(a.grad, a.grad_dtype, row);
    const float g = ppo_policy_dlp(lp, ps.olp, ps.A, ps.m, ps.inv_msum, a.cliprange, pt);
    if (threadIdx.x == 0) a.lp_out[row] = lp;
    return g;
}

// ------------------------------------------------------------------ rows that are not read
// Ragged batches.  A decoder position past its rollout's length (forward rows, `lengths`
// given) is store padding: the reference's collate pads each element's logprobs with 0.0
// (ppo_pipeline.py:47-65) and the GAE reads nothing past the length, so lp = 0 there and the
// row is not read.  A masked token of the loss (mask == 0) has dloss/dlp = 0 exactly (every
// path from lp to the loss is multiplied by the mask, ppo_models.py:165-177), so its dlogits
// row g·(onehot − p) is zeros, and lp reaches no other output: log_ratio = (lp − olp)·0 = 0
// for every finite lp, which the token record below uses with lp = 0 (lp_out = 0).  The
// row is written as zeros without being read.  (A masked row of non-finite logits made the
// reference's loss NaN through NaN·0; here it is not read at all — DESIGN.md §7.)  Both
// checks are block-uniform scalar loads ahead of the row; without lengths / mask the
// launches skip them.
__device__ __forceinline__ void pad_write(const RowArgs& a, int64_t row) {
    if (threadIdx.x == 0) {
        st_any(blockIdx.y == 0 ? a.lp0 : a.lp1, a.out_dtype, row, 0.0f);
        float* lse_out = blockIdx.y == 0 ? a.lse0 : a.lse1;
        if (lse_out) lse_out[row] = 0.0f;
    }
}
__device__ __forceinline__ bool pad_row(const RowArgs& a, int64_t row) {
    const int64_t b = row / a.T;
    if (row - b * a.T < a.lengths[b]) return false;
    pad_write(a, row);
    return true;
}

// Dispatch order of a ragged batch's forward rows: the valid rows (b, t < L_b) first, in row
// order, then the padding rows as ~row.  Measured (tools/ragged_probe.py): the same skipped
// rows cost ~20 us more at C3 when they are interleaved with the valid rows in dispatch order
// than when they come after them (a skipped workgroup's short life idles its slot), so the
// launch that takes its rows in this order pays this small launch instead (7.0 us with one
// workgroup, round 3's first form, profiles/r03i_c3_kernel_stats.txt).
// A grid of workgroups, each writing kOrderPos consecutive rows' entries (coalesced): every
// workgroup sums the clamped lengths itself (all of them, and those before its first rollout),
// scans its own rollouts' lengths in LDS, then places its rows — no pass over the batch by one
// workgroup, no per-thread run of T scattered stores (B·T < 2^31).
constexpr int kOrderThreads = 256;
constexpr int kOrderPos = 1024;  // rows per workgroup: at most kOrderPos + 1 rollouts
__device__ inline int order_wave_sum(int v) {
    for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off);
    return v;
}
__global__ __launch_bounds__(kOrderThreads) void k_ragged_order(const int64_t* lengths, int B, int T, int* order,
                                                                int* count) {
    __shared__ int s_len[kOrderPos + 1], s_vo[kOrderPos + 1];
    __shared__ int s_red[2][kOrderThreads / kWave], s_wsum[kOrderThreads / kWave];
    const int tid = threadIdx.x, lane = tid & (kWave - 1), w = tid / kWave;
    const int64_t n = int64_t(B) * T;
    const int64_t p0 = int64_t(blockIdx.x) * kOrderPos, p1 = min(p0 + kOrderPos, n);
    const int b0 = int(p0 / T), b1 = int((p1 - 1) / T) + 1, nb = b1 - b0;
    // the valid rows in all, and before rollout b0; this workgroup's rollouts' lengths to LDS
    int tot = 0, pre = 0;
    for (int b = tid; b < B; b += kOrderThreads) {
        const int Lb = int(min(max(lengths[b], int64_t(0)), int64_t(T)));
        tot += Lb;
        pre += b < b0 ? Lb : 0;
        if (b >= b0 && b < b1) s_len[b - b0] = Lb;
    }
    tot = order_wave_sum(tot);
    pre = order_wave_sum(pre);
    if (lane == 0) {
        s_red[0][w] = tot;
        s_red[1][w] = pre;
    }
    __syncthreads();
    int nvalid = 0, run = 0;
    for (int k = 0; k < kOrderThreads / kWave; ++k) {
        nvalid += s_red[0][k];
        run += s_red[1][k];
    }
    // exclusive scan of s_len: thread tid takes rollouts [tid·per, tid·per + per)
    const int per = (nb + kOrderThreads - 1) / kOrderThreads;
    const int i0 = min(nb, tid * per), i1 = min(nb, i0 + per);
    int loc = 0;
    for (int i = i0; i < i1; ++i) loc += s_len[i];
    int inc = loc;
    for (int off = 1; off < kWave; off <<= 1) {
        const int u = __shfl_up(inc, off);
        inc += lane >= off ? u : 0;
    }
    if (lane == kWave - 1) s_wsum[w] = inc;
    __syncthreads();
    for (int k = 0; k < w; ++k) run += s_wsum[k];
    run += inc - loc;
    for (int i = i0; i < i1; ++i) {
        s_vo[i] = run;  // valid rows before rollout b0 + i
        run += s_len[i];
    }
    __syncthreads();
    // row p = b·T + j: valid -> vo_b + j; padding -> after every valid row, in row order
    for (int64_t p = p0 + tid; p < p1; p += kOrderThreads) {
        const int b = int(p / T), j = int(p - int64_t(b) * T);
        const int Lb = s_len[b - b0], vo = s_vo[b - b0];
        if (j < Lb)
            order[vo + j] = int(p);
        else
            order[nvalid + (int(p) - j - vo) + (j - Lb)] = ~int(p);
    }
    if (blockIdx.x == 0 && tid == 0) *count = nvalid;  // after the list (trlx_ragged_order_bytes)
}

// Whether the mask can hold a zero: its sum (the launch's Σmask, one L2-resident scalar) short
// of B·T.  Only then does every row load its own mask element before its loads (that load
// cost the C3-shape loss rows ~6 us with an all-ones mask).  A sum that hides zeros behind
// weights > 1 only skips the skip — the rows are then computed, which is exact too.
__device__ __forceinline__ bool any_masked(const RowArgs& a) {
    const double msum = a.msum ? *a.msum : a.msum_host;
    return msum != double(a.B * a.T);
}

template <class DT>
__device__ __forceinline__ void masked_row(const RowArgs& a, int64_t row) {
    typedef typename DT::elem_t E;
    const int64_t b = row / a.T, t = row - b * a.T;
    E* drow = reinterpret_cast<E*>(a.dx) + b * a.dsb + t * a.dst;
    const RowSplit<DT> s(drow, a.V);  // the gradient row's own 16-B phase
    const int tid = threadIdx.x, nthr = blockDim.x;
    const __amdgpu_buffer_rsrc_t rout = make_rsrc(drow + s.head, uint32_t(s.nvec) * 16u);
    const vec4u z = {0u, 0u, 0u, 0u};
    for (int i = tid; i < int(s.nvec); i += nthr) store_grad_b128(z, rout, i * 16, a.spol);
    if (tid < s.head) DT::store1(drow, tid, 0.0f);
    if (tid < s.tail) DT::store1(drow, s.tail0 + tid, 0.0f);
    if (tid == 0) {
        float vin[3];
        const PpoScalars p = ppo_scalars(a, row, vin, true);
        PolicyTerms pt;
        ppo_policy_dlp(0.0f, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
        a.lp_out[row] = 0.0f;
        token_record(a, row, pt, p, vin);
        if (a.coef || a.wstats) split_outputs(a, row, p);
    }
}

// ------------------------------------------------------------------ register-resident rows
// SAME_PHASE: every dlogits row starts at the same address mod 16 as its logits row (the
// host checks strides and base phases; grad_buffer_like guarantees it), so dlogits are
// written with the same aligned 16-B vectors.  The other instantiation writes elements.
// LB512: launched with <= 512 threads, compiled for 8 waves per SIMD (64 VGPRs): the default
// for forward rows of <= 8 vectors per thread — T5 / UL2's V = 32128 bf16: four rows in flight
// per CU instead of three (C4 experience rows 312 -> 306 us, C3 235 -> 232 us; the folded loss
// tail's blocks spill a few doubles, the row path none) — and an opt-in knob elsewhere.
// NL > 0 (split residency, long fp32 rows): the row's last NL vector steps are DMA'd into
// LDS (32 KB per workgroup at NL = 4) instead of VGPRs, so a 512-thread workgroup fits in
// 128 VGPRs and two rows stay in flight per CU (a 201-KB fp32 row held whole in VGPRs
// needs 1024 threads at ~88 VGPRs: one row per CU, its load / reduce / store phases exposed).
// One row of the resident kernel (the workgroup's `row`).  MASKED (loss rows with a mask): the
// masked-token path is compiled in; the kernels of unmasked launches do not carry it (its
// inlined code measured 7-11 % slower rows at the C4 strong-scaling shape).
template <class DT, int NV, int MODE, bool SAME_PHASE, bool LB512, int NL, int WPE, bool MASKED>
__device__ __forceinline__ void vocab_row(const RowArgs& a, int64_t row) {
    __shared__ float sh_max[kMaxThreads / kWave];
    __shared__ float sh_max2[kMaxThreads / kWave];
    __shared__ float sh_sum[kMaxThreads / kWave];
    if constexpr (MODE == kFwd) {
        if (a.lengths && !a.row_list && pad_row(a, row)) return;
    }
    if constexpr (MODE == kPpo && MASKED) {
        if (any_masked(a) && a.mask[row] == 0) {
            masked_row<DT>(a, row);
            return;
        }
    }
    typedef typename DT::elem_t E;
    constexpr int EPV = DT::kEPV;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const Row<DT> r(a, row);
    // Row-independent scalars first, computed by thread 0 while the row loads are in
    // flight and parked in LDS (read back after the reductions' barriers): they then
    // occupy no VGPRs beside the row.
    __shared__ float s_ps[12];
    if (MODE == kPpo && tid == 0) {
        float vin[3];
        const PpoScalars p0 = ppo_scalars(a, r.row, vin, true);
        s_ps[0] = p0.A; s_ps[1] = p0.m; s_ps[2] = p0.inv_msum; s_ps[3] = p0.olp;
        if (a.tokrec) { s_ps[4] = vin[0]; s_ps[5] = vin[1]; s_ps[6] = vin[2]; }
        s_ps[7] = p0.beta; s_ps[8] = p0.mu; s_ps[9] = p0.rstd; s_ps[10] = p0.rew; s_ps[11] = p0.R;
    }

    const int nvec = int(r.s.nvec);
    const __amdgpu_buffer_rsrc_t rin = make_rsrc(r.x + r.s.head, uint32_t(nvec) * 16u);
    const int shift = line_shift(r.x + r.s.head);  // whole 256-B spans per wave instruction
    // Vector order (tuning "row_order"): 0 = step-major (vector tid + k*nthr), 1 = wave-major
    // (wave w owns the contiguous vectors [w*NT*64, (w+1)*NT*64), NT = NV + NL: its VGPR steps,
    // then its LDS steps); both issue one 1-KB span
    // per wave instruction.  Both strides are runtime values, so the per-vector offsets are
    // added in VOFFSET (the raw-buffer range check covers voffset + imm, not soffset): the
    // first `shift` lanes wrap to huge offsets at k = 0 and are dropped like those past the body.
    const int vbase = (a.order ? (tid >> 6) * ((NV + NL) * kWave) + (tid & (kWave - 1)) : tid) - shift;
    const int vstep = a.order ? kWave : nthr;
    const int voff = vbase * 16;
    // ---- one HBM read of the row into registers (all loads in flight at once).  Vectors
    // past the row body read 0 (range check) and are excluded per vector below.
    vec4u v[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k)
        v[k] = __builtin_amdgcn_raw_buffer_load_b128(rin, launder_int(voff) + k * vstep * 16, 0, kAuxNT);
    __shared__ __attribute__((aligned(16))) vec4u lds_row[NL > 0 ? NL * 512 : 1];
    if constexpr (NL > 0) {  // vector steps NV .. NV+NL-1 -> lds_row[kk][tid] (lane-linear per wave)
        const char* body = reinterpret_cast<const char*>(r.x + r.s.head);
        char* lbase = reinterpret_cast<char*>(lds_row) + (tid >> 6) * 1024;
#pragma unroll
        for (int kk = 0; kk < NL; ++kk) {
            const int i = vbase + (NV + kk) * vstep;
            const int ic = unsigned(i) < unsigned(nvec) ? i : 0;  // out-of-row lanes: any valid address
            __builtin_amdgcn_global_load_lds(body + int64_t(ic) * 16,
                                             (__attribute__((address_space(3))) void*)(lbase + kk * 8192), 16, 0, 0);
        }
    }
    const float xy = r.y_ok ? DT::load1(r.x, r.y) : NAN;
    const int64_t je = r.edge_index();
    const float ex = je >= 0 ? DT::load1(r.x, je) : -INFINITY;

    // lp = (x[y] - max) - log Σ exp(x - max), the reference's log_softmax order
    // (x - max first, exact for bf16 rows): xy - (max + log Σ) would lose the low bits of lp
    // to the rounding of lse when |max| is large.
    float lse, lp = 0.0f;
    if (MODE == kBwd) {
        lse = a.lse_in[r.row];
    } else {
        float m;
        bool exact = true;
        if constexpr (sizeof(E) == 2) {
            // Raw-bits maximum of bf16 rows, two elements per v_pk_max_i16 and no unpacking:
            // non-negative floats order like their bit patterns read as signed int16, negative
            // ones read as negative int16 below all of them, so for a row whose maximum is >= +0
            // the largest bit pattern IS the maximum (a lane holding only negatives reports a
            // wrong, smaller value, which cannot win).  Out-of-row lanes count as -0.0 (0x8000,
            // the smallest int16).  A row whose maximum comes out negative or -0.0 re-runs the
            // exact float pass below (block-uniform branch).  NaN / +-inf: +inf and positive
            // NaN bit patterns exceed every finite value, so m is +inf / NaN exactly when the
            // float pass would make lse NaN anyway.
            constexpr uint32_t kNeg0 = 0x80008000u;  // -0.0 in both halves: the smallest int16
            uint32_t acc = kNeg0;
#pragma unroll
            for (int k = 0; k < NV; ++k) {
                const uint32_t p = pk_max_i16(pk_max_i16(v[k].x, v[k].y), pk_max_i16(v[k].z, v[k].w));
                acc = pk_max_i16(acc, unsigned(vbase + k * vstep) < unsigned(nvec) ? p : kNeg0);
            }
            if constexpr (NL > 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's DMAs (it reads only its own)
#pragma unroll
                for (int kk = 0; kk < NL; ++kk) {
                    const vec4u w = lds_row[kk * 512 + tid];
                    const uint32_t p = pk_max_i16(pk_max_i16(w.x, w.y), pk_max_i16(w.z, w.w));
                    acc = pk_max_i16(acc, unsigned(vbase + (NV + kk) * vstep) < unsigned(nvec) ? p : kNeg0);
                }
            }
            const int mi = max(int(int16_t(acc & 0xffffu)), int(acc) >> 16);  // the two halves, sign-extended
            m = block_max(fmaxf(__uint_as_float(uint32_t(mi) << 16), ex), sh_max);
            exact = signbit(m) != 0;
#pragma unroll
            for (int k = 0; k < NV; ++k) launder(v[k]);
        }
        if (exact) {
        m = ex;
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[EPV];
            DT::unpack(v[k], f);
            float mk = f[0];
#pragma unroll
            for (int e = 1; e < EPV; ++e) mk = fmaxf(mk, f[e]);
            m = (unsigned(vbase + k * vstep) < unsigned(nvec)) ? fmaxf(m, mk) : m;
        }
        if constexpr (NL > 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this lane's DMAs (it reads only its own)
#pragma unroll
            for (int kk = 0; kk < NL; ++kk) {
                float f[EPV];
                DT::unpack(lds_row[kk * 512 + tid], f);
                float mk = f[0];
#pragma unroll
                for (int e = 1; e < EPV; ++e) mk = fmaxf(mk, f[e]);
                m = (unsigned(vbase + (NV + kk) * vstep) < unsigned(nvec)) ? fmaxf(m, mk) : m;
            }
        }
        m = block_max(m, sh_max2);
        }
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        const float ml2e = -m * kLog2e;
        const f32x2 l2e2 = f2_splat(kLog2e), ml2e2 = f2_splat(ml2e), zero2 = f2_splat(0.0f);
        // element pairs: v_pk_fma_f32 scale, v_exp_f32 per element, v_pk_add_f32 accumulate
        f32x2 acc = {exp2_fast(fmaf(ex, kLog2e, ml2e)), 0.0f};
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            float f[EPV];
            DT::unpack(v[k], f);
            const f32x2 sk = exp_pair_sum(f, l2e2, ml2e2);
            acc += (unsigned(vbase + k * vstep) < unsigned(nvec)) ? sk : zero2;
        }
        if constexpr (NL > 0) {
#pragma unroll
            for (int kk = 0; kk < NL; ++kk) {
                float f[EPV];
                DT::unpack(lds_row[kk * 512 + tid], f);
                const f32x2 sk = exp_pair_sum(f, l2e2, ml2e2);
                acc += (unsigned(vbase + (NV + kk) * vstep) < unsigned(nvec)) ? sk : zero2;
            }
        }
        float sum = acc.x + acc.y;
        sum = block_sum(sum, sh_sum);
#pragma unroll
        for (int k = 0; k < NV; ++k) launder(v[k]);
        // The exponent offset ml2e = -m·log2e is rounded: each term above is 2^((x - m)·log2e + d)
        // with d = m·log2e + ml2e, the exact residual of that product (fma, TwoProduct).  Undo
        // it once per row (it is up to ~5e-4 at |m| ~ 1e4, far above the lp tolerance).
        const float d = isfinite(m) ? fmaf(m, kLog2e, ml2e) : 0.0f;
        const float lsum = logf(sum) - d * kLn2;
        lse = m + lsum;
        lp = (xy - m) - lsum;
    }
    if (MODE == kFwd) {
        fwd_epilogue(a, r, lp, lse);
        return;
    }

    if constexpr (NL > 0) {
        if (MODE == kBwd) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no reduction pass waited
    }
    // (both reductions' barriers separate thread 0's s_ps writes from these reads)
    const PpoScalars ps = {s_ps[0], s_ps[1], s_ps[2], s_ps[3]};
    PolicyTerms pt = {1.f, 0.f, 0.f, false};
    const float g = row_grad<MODE>(a, r.row, lp, ps, pt);

    // ---- dlogits = g * (onehot(y) - exp(x - lse)), written once
    const float lse_l2e = -lse * kLog2e;
    // as for the sum: 2^(x·log2e + lse_l2e) = p(x) · 2^d2, d2 the residual of the rounded
    // offset; the per-row factor 2^-d2 rides on g
    const float corr = isfinite(lse) ? exp2_fast(-fmaf(lse, kLog2e, lse_l2e)) : 1.0f;
    const float ng = -g * corr;
    E* drow = reinterpret_cast<E*>(a.dx) + r.b * a.dsb + r.t * a.dst;
    const float gy = g * (1.0f - corr * exp2_fast(fmaf(xy, kLog2e, lse_l2e)));
    // edge elements first, and the token record's inputs parked in LDS (thread 0 reads them
    // back after the loop): fewer values live beside the row during the store loop
    if (je >= 0) DT::store1(drow, je, je == r.y ? gy : ng * exp2_fast(fmaf(ex, kLog2e, lse_l2e)));
    __shared__ float s_tok[6];
    if (MODE == kPpo && tid == 0) {
        s_tok[0] = pt.ratio; s_tok[1] = pt.lr; s_tok[2] = pt.pgmax; s_tok[3] = pt.pgclip ? 1.f : 0.f;
        s_tok[4] = ps.m; s_tok[5] = ps.inv_msum;
    }
    if (SAME_PHASE) {
        const __amdgpu_buffer_rsrc_t rout = make_rsrc(drow + r.s.head, uint32_t(nvec) * 16u);
        const int iy = r.y_ok && r.y >= r.s.head && r.y < r.s.tail0 ? int((r.y - r.s.head) / EPV) : -1;
        const f32x2 l2e2 = f2_splat(kLog2e), c2 = f2_splat(lse_l2e), ng2 = f2_splat(ng);
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int i = vbase + k * vstep;  // lanes outside the body: range-checked away
            float f[EPV];
            DT::unpack(v[k], f);
            neg_g_exp_pairs(f, l2e2, c2, ng2);
            if (i == iy) {  // the label's vector: onehot term
                const int ey = int(r.y - (r.s.head + int64_t(i) * EPV));
#pragma unroll
                for (int e = 0; e < EPV; ++e)
                    if (e == ey) f[e] = gy;
            }
            const vec4u pk = DT::pack(f);
            const int off = launder_int(voff) + k * vstep * 16;
            store_grad_b128(pk, rout, off, a.spol);
        }
        if constexpr (NL > 0) {
#pragma unroll
            for (int kk = 0; kk < NL; ++kk) {
                const int i = vbase + (NV + kk) * vstep;
                float f[EPV];
                DT::unpack(lds_row[kk * 512 + tid], f);
                neg_g_exp_pairs(f, l2e2, c2, ng2);
                if (i == iy) {
                    const int ey = int(r.y - (r.s.head + int64_t(i) * EPV));
#pragma unroll
                    for (int e = 0; e < EPV; ++e)
                        if (e == ey) f[e] = gy;
                }
                __builtin_amdgcn_raw_buffer_store_b128(DT::pack(f), rout, launder_int(voff) + (NV + kk) * vstep * 16, 0,
                                                       kAuxNT);
            }
        }
    } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
            const int i = vbase + k * vstep;
            if (unsigned(i) < unsigned(nvec)) {
                float f[EPV];
                DT::unpack(v[k], f);
#pragma unroll
                for (int e = 0; e < EPV; ++e) {
                    const int64_t j = r.s.head + int64_t(i) * EPV + e;
                    DT::store1(drow, j, j == r.y ? gy : ng * exp2_fast(fmaf(f[e], kLog2e, lse_l2e)));
                }
            }
        }
        if constexpr (NL > 0) {
#pragma unroll
            for (int kk = 0; kk < NL; ++kk) {
                const int i = vbase + (NV + kk) * vstep;
                if (unsigned(i) < unsigned(nvec)) {
                    float f[EPV];
                    DT::unpack(lds_row[kk * 512 + tid], f);
#pragma unroll
                    for (int e = 0; e < EPV; ++e) {
                        const int64_t j = r.s.head + int64_t(i) * EPV + e;
                        DT::store1(drow, j, j == r.y ? gy : ng * exp2_fast(fmaf(f[e], kLog2e, lse_l2e)));
                    }
                }
            }
        }
    }
    if (MODE == kPpo && tid == 0) {
        const PolicyTerms t2 = {s_tok[0], s_tok[1], s_tok[2], s_tok[3] != 0.f};
        const PpoScalars p2 = {0.f, s_tok[4], s_tok[5], 0.f, s_ps[7], s_ps[8], s_ps[9], s_ps[10], s_ps[11]};
        token_record(a, r.row, t2, p2, s_ps + 4);
        if (a.coef || a.wstats) split_outputs(a, r.row, p2);
    }
}

template <class DT, int NV, int MODE, bool SAME_PHASE, bool LB512, int NL = 0, int WPE = 4, bool MASKED = false>
__global__ __launch_bounds__((LB512 || NL) ? 512 : kMaxThreads, LB512 ? 8 : (NL ? WPE : 1)) void k_vocab_rows(RowArgs a) {
    if constexpr (MODE == kFwd) {
        if (int(blockIdx.x) < a.tail_blocks) {  // the previous step's loss tail (block-uniform branch)
            __shared__ double tail_red[kMaxThreads / kWave * 16];
            if (blockIdx.y == 0) loss_tail_block(a.tail, int(blockIdx.x), a.tail_blocks, tail_red);
            return;
        }
    }
    if constexpr (MODE == kPpo && NL > 0) {  // only the split-residency kernels host it (their VGPR
                                             // budget is set by the row; the others run it standalone)
        if (int(blockIdx.x) < a.gae_blocks) {  // the next batch's split GAE (block-uniform branch)
            __shared__ double gae_red[kMaxThreads / kWave * 8];
            gae_block<true>(a.gae, int(blockIdx.x), a.gae_blocks, gae_red);
            return;
        }
    }
    int64_t row = int64_t(blockIdx.x) - a.lead_blocks;
    if constexpr (MODE == kFwd) {
        if (a.row_list) {  // a ragged batch in valid-rows-first order
            const int r = a.row_list[row];
            if (r < 0) {
                pad_write(a, ~int64_t(r));
                return;
            }
            row = r;
        }
    }
    vocab_row<DT, NV, MODE, SAME_PHASE, LB512, NL, WPE, MASKED>(a, row);
}

// ------------------------------------------------------------------ streaming rows
// Same arithmetic, but the row is streamed through registers U vectors at a time with an
// online (max, sum-exp) instead of being held whole: small register footprint => many
// workgroups per CU keep loads continuously in flight.  Backward / fused modes make a
// second pass over the row (served from L2 / the Infinity Cache when it was just read).
__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
    const float nm = fmaxf(m, m2);
    if (nm == -INFINITY) return;  // both empty
    s = s * exp2_fast((m - nm) * kLog2e) + s2 * exp2_fast((m2 - nm) * kLog2e);
    m = nm;
}

constexpr int kStreamMaxThreads = 256;  // launch bound of the streaming kernel (register budget)

template <class DT, int U, int MODE>
__global__ __launch_bounds__(kStreamMaxThreads) void k_vocab_rows_stream(RowArgs a) {
    __shared__ float sh_m[kStreamMaxThreads / kWave];
    __shared__ float sh_s[kStreamMaxThreads / kWave];
    if constexpr (MODE == kFwd) {
        if (a.lengths && pad_row(a, int64_t(blockIdx.x))) return;
    }
    if constexpr (MODE == kPpo) {
        if (a.mask && any_masked(a) && a.mask[blockIdx.x] == 0) {
            masked_row<DT>(a, int64_t(blockIdx.x));
            return;
        }
    }
    typedef typename DT::elem_t E;
    constexpr int EPV = DT::kEPV;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const Row<DT> r(a);
    PpoScalars ps = {0.f, 1.f, 1.f, 0.f};
    float vin[3];
    if (MODE == kPpo) ps = ppo_scalars(a, r.row, vin, false);
    const vec4u* vp = reinterpret_cast<const vec4u*>(r.x + r.s.head);
    const int64_t nvec = r.s.nvec;
    const int64_t je = r.edge_index();
    const float ex = je >= 0 ? DT::load1(r.x, je) : -INFINITY;

    float lse, lsum = 0.0f, mx = 0.0f;  // kBwd: lse given, lp unused
    if (MODE == kBwd) {
        lse = a.lse_in[r.row];
    } else {
        float m = ex, sum = (ex == -INFINITY) ? 0.0f : 1.0f;
        for (int64_t base = tid; base < nvec; base += int64_t(nthr) * U) {
            vec4u v[U];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int64_t i = base + int64_t(u) * nthr;
                v[u] = (i < nvec) ? ld_stream(vp + i) : DT::neg_inf();
            }
            float mx = -INFINITY;
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float f[EPV];
                DT::unpack(v[u], f);
#pragma unroll
                for (int e = 0; e < EPV; ++e) mx = fmaxf(mx, f[e]);
            }
#pragma unroll
            for (int u = 0; u < U; ++u) launder(v[u]);
            const float nm = fmaxf(m, mx);
            if (nm == -INFINITY) continue;
            sum *= exp2_fast((m - nm) * kLog2e);
            const float nml2e = -nm * kLog2e;
            f32x2 acc = {0.0f, 0.0f};  // packed pairs (v_pk_fma_f32 / v_pk_add_f32)
#pragma unroll
            for (int u = 0; u < U; ++u) {
                float f[EPV];
                DT::unpack(v[u], f);
                acc += exp_pair_sum(f, f2_splat(kLog2e), f2_splat(nml2e));
            }
            // this chunk's terms carry 2^d, d the residual of the rounded offset (see k_vocab_rows)
            sum += (acc.x + acc.y) * exp2_fast(-fmaf(nm, kLog2e, nml2e));
            m = nm;
        }
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const float m2 = __shfl_xor(m, off, kWave), s2 = __shfl_xor(sum, off, kWave);
            online_merge(m, sum, m2, s2);
        }
        if ((tid & (kWave - 1)) == 0) {
            sh_m[tid / kWave] = m;
            sh_s[tid / kWave] = sum;
        }
        __syncthreads();
        m = sh_m[0];
        sum = sh_s[0];
        for (int w = 1; w < nthr / kWave; ++w) online_merge(m, sum, sh_m[w], sh_s[w]);
        lsum = logf(sum);
        lse = m + lsum;
        mx = m;
    }
    const float xy = r.y_ok ? DT::load1(r.x, r.y) : NAN;
    const float lp = (xy - mx) - lsum;  // the reference's order, as in k_vocab_rows
    if (MODE == kFwd) {
        fwd_epilogue(a, r, lp, lse);
        return;
    }
    PolicyTerms pt = {1.f, 0.f, 0.f, false};
    const float g = row_grad<MODE>(a, r.row, lp, ps, pt);
    const float lse_l2e = -lse * kLog2e;
    const float corr = isfinite(lse) ? exp2_fast(-fmaf(lse, kLog2e, lse_l2e)) : 1.0f;  // as in k_vocab_rows
    const float ng = -g * corr;
    E* drow = reinterpret_cast<E*>(a.dx) + r.b * a.dsb + r.t * a.dst;
    const float gy = g * (1.0f - corr * exp2_fast(fmaf(xy, kLog2e, lse_l2e)));
    const bool same_phase = ((reinterpret_cast<uintptr_t>(drow) ^ reinterpret_cast<uintptr_t>(r.x)) & 15u) == 0;
    const int64_t iy = r.y_ok && r.y >= r.s.head && r.y < r.s.tail0 ? (r.y - r.s.head) / EPV : -1;
    vec4u* dvp = reinterpret_cast<vec4u*>(drow + r.s.head);
    for (int64_t base = tid; base < nvec; base += int64_t(nthr) * U) {
        vec4u v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + int64_t(u) * nthr;
            if (i < nvec) v[u] = vp[i];  // second touch: cached read
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int64_t i = base + int64_t(u) * nthr;
            if (i >= nvec) continue;
            float f[EPV];
            DT::unpack(v[u], f);
            neg_g_exp_pairs(f, f2_splat(kLog2e), f2_splat(lse_l2e), f2_splat(ng));
            if (same_phase) {
                if (i == iy) {
                    const int ey = int(r.y - (r.s.head + i * EPV));
#pragma unroll
                    for (int e = 0; e < EPV; ++e)
                        if (e == ey) f[e] = gy;
                }
                __builtin_nontemporal_store(DT::pack(f), dvp + i);
            } else {
#pragma unroll
                for (int e = 0; e < EPV; ++e) {
                    const int64_t j = r.s.head + i * EPV + e;
                    DT::store1(drow, j, j == r.y ? gy : f[e]);
                }
            }
        }
    }
    if (je >= 0) DT::store1(drow, je, je == r.y ? gy : ng * exp2_fast(fmaf(ex, kLog2e, lse_l2e)));
    if (MODE == kPpo && a.tokrec && tid == 0) {
        PpoScalars p2 = ps;
        if (a.coef || a.wstats)
            split_value_inputs(a, r.row, split_advantage(a, r.row, ps.beta), vin, p2.R);
        else
            loss_token_inputs(a.ltok, r.row, vin);
        token_record(a, r.row, pt, ps, vin);
        if (a.coef || a.wstats) split_outputs(a, r.row, p2);
    }
}

// ------------------------------------------------------------------ launch geometry
struct Geometry {
    int nv;
    int threads;
};

// Tuning knobs (trlx_set_tuning): 0 = automatic.
static TuneKnob g_row_variant{0};       // 1 = register-resident rows, 2 = streaming rows
static TuneKnob g_resident_threads{0};  // preferred workgroup size for resident rows
static TuneKnob g_resident_lb512{0};    // 1 = <=512-thread rows compiled for 8 waves/SIMD
static TuneKnob g_stream_threads{0};
static TuneKnob g_stream_unroll{0};
static TuneKnob g_row_order{0};         // resident rows: 0 = step-major vectors, 1 = wave-major
static TuneKnob g_ragged_order{0};      // forward rows with lengths: 0 auto (valid rows first), 1 natural
static TuneKnob g_order_launch{0};  // ragged order: 0 auto, 1 one launch (k_ragged_order), 2 two (row_order.h)
static TuneKnob g_store_pol{0};         // gradient-row stores: 0 auto, 1 none, 2 sc1, 3 sc0|sc1, 4 nt|sc1, 5 nt
constexpr double kSC1Bytes = 1.5e9;  // auto: sc1 above this many gradient bytes per launch, else nt

// Cache policy of a launch's gradient-row stores (common.h store_grad_b128).  Measured
// (tools/policy_sweep.py, interleaved): sc1 wins on the all-VGPR rows kernel once a launch
// writes more than ~1.5 GB (V = 32128 bf16: +1 % at 1.6 GB, +5 % at 8.4 GB) and loses on the
// split-residency kernels at every size (V = 50257: -4 % at 1.9 / 2.5 GB) and below 1 GB.
static int store_policy_for(double grad_bytes, bool split) {
    if (g_store_pol == 5) return kStoreNT;
    if (g_store_pol) return g_store_pol;
    return (!split && grad_bytes > kSC1Bytes) ? kStoreSC1 : kStoreNT;
}
static TuneKnob g_split_lds{0};         // long rows: 0 auto (split LDS + VGPR residency), 1 off, 2 also forward
static TuneKnob g_split_mid{0};         // mid bf16 rows (loss / backward): 0 auto (= 3), 1 off, 2 5+3, 3 6+2
int tuning_split_lds() { return g_split_lds; }
static TuneKnob g_ilql_split{0};  // ILQL fp32 split residency: 0 = 20 VGPR + 5 LDS steps, 1 = 22 + 3, 2 = 21 + 4, 3 = 19 + 6
int tuning_ilql_split() { return g_ilql_split; }

// Register-resident geometry: NV (compile-time vectors per thread, from kNVs) and the
// workgroup size.  Default: 512-thread workgroups (8 waves) -- measured on MI355X (C2,
// bf16 V=50257): 3 rows in flight per CU at ~71 VGPRs, 6.6-6.7 TB/s for the forward;
// rows too long for 16 vectors x 512 threads use 1024 threads (backward / fused) or the
// streaming kernel (forward: measured faster than 1024-thread resident rows).
static const int kNVs[] = {1, 2, 3, 4, 5, 6, 7, 8, 10, 12, 13, 16};

static Geometry pick_geometry(int64_t V, int elem_bytes, bool allow_1024) {
    const int epv = 16 / elem_bytes;
    const int64_t nvec = V / epv + 1 + (kLineVecs - 1);  // upper bound incl. peeling and line shift
    const int prefs[2] = {g_resident_threads > 0 ? g_resident_threads : 512, kMaxThreads};
    for (int pi = 0; pi < (allow_1024 ? 2 : 1); ++pi) {
        const int pref = prefs[pi];
        const int64_t need = (nvec + pref - 1) / pref;
        for (int nv : kNVs) {
            if (nv < need) continue;
            int64_t thr = (nvec + nv - 1) / nv;
            thr = ((thr + kWave - 1) / kWave) * kWave;
            return {nv, int(thr < kWave ? kWave : thr)};
        }
        if (g_resident_threads > 0) break;  // a fixed size that does not fit -> streaming
    }
    return {0, 0};
}

// True when every dlogits row (b, t) has the same 16-byte phase as its logits row.
static bool rows_same_phase(const RowArgs& a, size_t es) {
    if (!a.dx) return true;
    const bool same_steps = (a.B <= 1 || ((a.sb - a.dsb) * int64_t(es)) % 16 == 0) &&
                            (a.T <= 1 || ((a.st - a.dst) * int64_t(es)) % 16 == 0);
    return same_steps && ((reinterpret_cast<uintptr_t>(a.x0) ^ reinterpret_cast<uintptr_t>(a.dx)) & 15u) == 0;
}

// Rows launch with the launch's done event (hipExtLaunchKernel stop event) when one is set.
#define TRLX_ROWS_LAUNCH(KERN, GRID, BLOCK, STREAM, A)                                                        \
    do {                                                                                                     \
        if ((A).done_event)                                                                                  \
            hipExtLaunchKernelGGL(KERN, GRID, BLOCK, 0, STREAM, nullptr, (hipEvent_t)(A).done_event, 0, A);  \
        else                                                                                                 \
            hipLaunchKernelGGL(KERN, GRID, BLOCK, 0, STREAM, A);                                             \
    } while (0)

// Resident rows launch: loss rows with a mask take the MASKED instantiation.
#define TRLX_RESIDENT_LAUNCH(DTX, NVX, SPX, LBX, NLX, WPEX, GRID, BLOCK, STREAM, A)                                    \
    do {                                                                                                         \
        if (MODE == kPpo && (A).mask)                                                                            \
            TRLX_ROWS_LAUNCH((k_vocab_rows<DTX, NVX, MODE, SPX, LBX, NLX, WPEX, MODE == kPpo>), GRID, BLOCK, STREAM, A); \
        else                                                                                                     \
            TRLX_ROWS_LAUNCH((k_vocab_rows<DTX, NVX, MODE, SPX, LBX, NLX, WPEX, false>), GRID, BLOCK, STREAM, A);  \
    } while (0)

// Work folded in ahead of the rows that a kernel cannot host runs as its own launch first:
// the loss tail (any resident kernel hosts it), the split GAE (hosted by workgroups of at
// least kRolloutThreads threads; never by the streaming rows).
static int lead_standalone(RowArgs& a, hipStream_t stream, bool tail, bool gae) {
    if (tail && a.has_tail) {
        a.has_tail = 0;
        const unsigned nblk = unsigned((a.tail.B + kRolloutsPerBlock - 1) / kRolloutsPerBlock);
        hipLaunchKernelGGL(k_rollout_loss, dim3(nblk), dim3(kRolloutThreads), 0, stream, a.tail);
        const int rc = check_launch("k_rollout_loss");
        if (rc) return rc;
    }
    if (gae && a.has_gae) {
        a.has_gae = 0;
        const unsigned nblk = unsigned((a.gae.B + kRolloutsPerBlock - 1) / kRolloutsPerBlock);
        hipLaunchKernelGGL(k_rollout_gae<true>, dim3(nblk), dim3(kRolloutThreads), 0, stream, a.gae);
        const int rc = check_launch("k_rollout_gae");
        if (rc) return rc;
    }
    return TRLX_OK;
}

// Leading workgroups of a rows launch of `threads`-wide workgroups: a folded loss tail needs
// one per (threads / 64) rollouts, a folded GAE one per 4 rollouts (split-residency kernels
// only: `split`).
static int rows_grid(RowArgs& a, int threads, int nten, hipStream_t stream, dim3& grid, bool split) {
    const int rc = lead_standalone(a, stream, false, !split || threads < kRolloutThreads);
    if (rc) return rc;
    a.tail_blocks = a.has_tail ? int((a.tail.B + threads / kWave - 1) / (threads / kWave)) : 0;
    a.gae_blocks = a.has_gae ? int((a.gae.B + kRolloutsPerBlock - 1) / kRolloutsPerBlock) : 0;
    a.lead_blocks = a.tail_blocks + a.gae_blocks;
    grid = dim3(unsigned(a.B * a.T + a.lead_blocks), unsigned(nten));
    return TRLX_OK;
}

template <int MODE, class DT>
static int launch_rows_dt(const RowArgs& a0, int nten, hipStream_t stream) {
    RowArgs a = a0;
    a.order = g_row_order;
    const double grad_bytes = double(a.B) * double(a.T) * double(a.V) * double(sizeof(typename DT::elem_t));
    a.spol = MODE == kFwd ? kStoreNT : store_policy_for(grad_bytes, true);  // split launches: LDS part nt
    if constexpr (sizeof(typename DT::elem_t) == 2) {
        // long bf16 rows (V > 32 k): 9 vectors per thread in VGPRs + 4 in LDS, 512 threads at
        // <= 85 VGPRs -> three rows in flight per CU instead of two (C2 loss row 2.9 % faster)
        const int64_t nvec = a.V / 8 + 1 + (kLineVecs - 1);
        const bool want = g_split_lds == 2 || (g_split_lds == 0 && MODE != kFwd);
        if (want && !g_row_variant && !g_resident_threads && nvec > 512 * 8 && nvec <= 512 * (9 + 4)) {
            dim3 grid;
            const int rc = rows_grid(a, 512, nten, stream, grid, true);
            if (rc) return rc;
            if (MODE == kFwd || rows_same_phase(a, 2))
                TRLX_RESIDENT_LAUNCH(DT, 9, true, false, 4, 6, grid, dim3(512), stream, a);
            else
                TRLX_RESIDENT_LAUNCH(DT, 9, false, false, 4, 6, grid, dim3(512), stream, a);
            return check_launch("k_vocab_rows (split LDS, bf16)");
        }
        // mid-length bf16 rows (V 16k-32k, T5/UL2's 32128) in the loss / backward: the last
        // vector steps in LDS as well, so the row kernel fits 64 VGPRs and FOUR rows are in
        // flight per CU (8 waves/SIMD) instead of three (tuning "split_mid": 1 off, 2 = 5 VGPR
        // + 3 LDS steps, 3 = 6 + 2, the default: measured C4 loss rows 363 -> 341 us, C3
        // 274 -> 247 us; 5 + 3 did not gain, profiles/r02_split_mid.log)
        // Auto only below kSC1Bytes of gradient rows per launch: past it the all-VGPR kernel's
        // `sc1` stores win (C4 at 1024 rollouts, 4.2 GB: 2.70 ms with them vs 2.91 ms split + nt).
        const int sm = g_split_mid ? g_split_mid : (grad_bytes > kSC1Bytes && !g_store_pol ? 1 : 3);
        if (MODE != kFwd && sm > 1 && g_split_lds != 1 && !g_row_variant && !g_resident_threads &&
            nvec > 512 * 4 && nvec <= 512 * 8 && rows_same_phase(a, 2)) {
            dim3 grid;
            const int rc = rows_grid(a, 512, nten, stream, grid, true);
            if (rc) return rc;
            if (sm == 3)
                TRLX_RESIDENT_LAUNCH(DT, 6, true, false, 2, 8, grid, dim3(512), stream, a);
            else
                TRLX_RESIDENT_LAUNCH(DT, 5, true, false, 3, 8, grid, dim3(512), stream, a);
            return check_launch("k_vocab_rows (split LDS, mid bf16)");
        }
    }
    if constexpr (sizeof(typename DT::elem_t) == 4) {
        // long fp32 rows: 21 vectors per thread in VGPRs + 4 in LDS, 512 threads, 2 rows per CU
        const int64_t nvec = a.V / 4 + 1 + (kLineVecs - 1);
        const bool want = g_split_lds == 2 || (g_split_lds == 0 && MODE != kFwd);
        if (want && !g_row_variant && !g_resident_threads && nvec > 512 * 16 && nvec <= 512 * (21 + 4)) {
            dim3 grid;
            const int rc = rows_grid(a, 512, nten, stream, grid, true);
            if (rc) return rc;
            if (MODE == kFwd || rows_same_phase(a, 4))
                TRLX_RESIDENT_LAUNCH(DT, 21, true, false, 4, 4, grid, dim3(512), stream, a);
            else
                TRLX_RESIDENT_LAUNCH(DT, 21, false, false, 4, 4, grid, dim3(512), stream, a);
            return check_launch("k_vocab_rows (split LDS)");
        }
    }
    a.spol = MODE == kFwd ? kStoreNT : store_policy_for(grad_bytes, false);
    const Geometry g = pick_geometry(a.V, sizeof(typename DT::elem_t), MODE != kFwd || g_resident_threads > 0);
    const int variant = g_row_variant ? g_row_variant : (g.nv > 0 ? 1 : 2);
    if (variant == 2 || g.nv == 0) {
        const int rc = lead_standalone(a, stream, true, true);
        if (rc) return rc;
        a.tail_blocks = a.gae_blocks = a.lead_blocks = 0;
        const dim3 grid(unsigned(a.B * a.T), unsigned(nten));
        const int thr = g_stream_threads ? g_stream_threads : kStreamMaxThreads;
        // fp32 forward (the GPT path's experience rows): 2 vectors per thread in flight per
        // step measured 1.3 % faster than 4 (C2 fp32 383 vs 387 us, scripts/r03_fp32_fwd_sweep.sh)
        const int unroll = g_stream_unroll ? g_stream_unroll : (MODE == kFwd && sizeof(typename DT::elem_t) == 4 ? 2 : 4);
        if (unroll == 8)
            TRLX_ROWS_LAUNCH((k_vocab_rows_stream<DT, 8, MODE>), grid, dim3(thr), stream, a);
        else if (unroll == 2)
            TRLX_ROWS_LAUNCH((k_vocab_rows_stream<DT, 2, MODE>), grid, dim3(thr), stream, a);
        else
            TRLX_ROWS_LAUNCH((k_vocab_rows_stream<DT, 4, MODE>), grid, dim3(thr), stream, a);
        return check_launch("k_vocab_rows_stream");
    }
    const bool same = MODE == kFwd || rows_same_phase(a, sizeof(typename DT::elem_t));
    const bool lb512 = g.threads <= 512 && (g_resident_lb512 || (MODE == kFwd && g.nv <= 8));
    if (MODE == kFwd && a.lengths && a.order_ws && !g_ragged_order) {  // valid rows first
        const int orc = launch_ragged_order(a.lengths, a.B, a.T, a.order_ws, stream);
        if (orc) return orc;
        a.row_list = a.order_ws;
    }
    const dim3 block(g.threads);
    dim3 grid;
    const int rc = rows_grid(a, g.threads, nten, stream, grid, false);
    if (rc) return rc;
#define TRLX_RESIDENT_CASE(N)                                                                          \
    case N:                                                                                           \
        if (same && lb512)                                                                            \
            TRLX_RESIDENT_LAUNCH(DT, N, true, true, 0, 4, grid, block, stream, a);   \
        else if (same)                                                                                \
            TRLX_RESIDENT_LAUNCH(DT, N, true, false, 0, 4, grid, block, stream, a);  \
        else                                                                                          \
            TRLX_RESIDENT_LAUNCH(DT, N, MODE == kFwd, false, 0, 4, grid, block, stream, a); \
        break;
    switch (g.nv) {
        TRLX_RESIDENT_CASE(1) TRLX_RESIDENT_CASE(2) TRLX_RESIDENT_CASE(3) TRLX_RESIDENT_CASE(4)
        TRLX_RESIDENT_CASE(5) TRLX_RESIDENT_CASE(6) TRLX_RESIDENT_CASE(7) TRLX_RESIDENT_CASE(8)
        TRLX_RESIDENT_CASE(10) TRLX_RESIDENT_CASE(12) TRLX_RESIDENT_CASE(13) TRLX_RESIDENT_CASE(16)
        default: TRLX_REQUIRE(false, TRLX_ERR_SHAPE, "no resident geometry for NV=%d", g.nv);
    }
#undef TRLX_RESIDENT_CASE
    return check_launch("k_vocab_rows");
}

template <int MODE>
static int launch_rows(const RowArgs& a, int dtype, int nten, hipStream_t stream) {
    if (a.B * a.T == 0) return TRLX_OK;
    if (dtype == TRLX_BF16) return launch_rows_dt<MODE, BF16T>(a, nten, stream);
    return launch_rows_dt<MODE, F32T>(a, nten, stream);
}

static int check_rows(const RowArgs& a, int dtype) {
    TRLX_REQUIRE(dtype == TRLX_F32 || dtype == TRLX_BF16, TRLX_ERR_DTYPE, "logits dtype %d unsupported", dtype);
    TRLX_REQUIRE(a.B >= 0 && a.T >= 0 && a.V > 0, TRLX_ERR_SHAPE, "bad shape B=%lld T=%lld V=%lld",
                 (long long)a.B, (long long)a.T, (long long)a.V);
    TRLX_REQUIRE(a.B * a.T <= 0x7fffffffLL, TRLX_ERR_SHAPE, "too many rows");
    TRLX_REQUIRE(a.V * 16 < (1LL << 32), TRLX_ERR_SHAPE, "vocab too large");
    TRLX_REQUIRE(a.x0 && a.labels, TRLX_ERR_ARG, "NULL logits/labels");
    return TRLX_OK;
}

// Workspace carve-up (16-B aligned sections), shared by both fused launches.
static size_t ws_align(size_t x) { return (x + 15) & ~size_t(15); }
static size_t carve_workspace(void* base, int64_t B, int64_t T, Workspace* w) {
    char* p = static_cast<char*>(base);
    const int64_t nblk = (B + kRolloutsPerBlock - 1) / kRolloutsPerBlock;
    size_t off = 0;
    if (w) w->tickets = reinterpret_cast<unsigned*>(p + off);
    off += 16;
    if (w) w->gae_rec = reinterpret_cast<double*>(p + off);
    off += ws_align(sizeof(double) * 8 * size_t(nblk));  // split-beta records are 8 wide
    if (w) w->loss_rec = reinterpret_cast<double*>(p + off);
    off += ws_align(sizeof(double) * 16 * size_t(nblk));
    if (w) w->tokrec = reinterpret_cast<float*>(p + off);
    off += ws_align(sizeof(float) * kTokRec * size_t(B * T));
    if (w) w->order = reinterpret_cast<int*>(p + off);
    off += ws_align(size_t(ragged_order_bytes(B, T)));
    return off;
}

size_t carve_ppo_workspace(void* base, int64_t B, int64_t T, Workspace* w) { return carve_workspace(base, B, T, w); }

int lmloss_set_tuning(const char* key, int64_t value, bool* handled);  // lmhead_loss.hip

// One launch while its workgroups' passes over all B lengths stay small (each reads every
// length: O(B²·T / 1024) loads in all — 12 x 256 at C3); past kOrderOneLaunchChunks the two
// chunk-count launches of row_order.h (O(B·T / 1024) loads per workgroup).
constexpr int64_t kOrderOneLaunchChunks = 64;
int launch_ragged_order(const int64_t* lengths, int64_t B, int64_t T, int* order, hipStream_t stream) {
    if (B * T == 0) return TRLX_OK;
    const int64_t nchunk = (B * T + kOrderPos - 1) / kOrderPos;
    if (g_order_launch == 2 || (g_order_launch == 0 && nchunk > kOrderOneLaunchChunks))
        return launch_order<true>(lengths, int(T), B * T, order + B * T + 4, order, stream);
    hipLaunchKernelGGL(k_ragged_order, dim3(unsigned(nchunk)), dim3(kOrderThreads), 0, stream, lengths, int(B),
                       int(T), order, order + B * T);
    return check_launch("k_ragged_order");
}

}  // namespace trlx

using namespace trlx;

extern "C" int trlx_lsm_gather_fwd(const void* x0, const void* x1, int dtype, int64_t B, int64_t T,
                                   int64_t V, int64_t sb, int64_t st, const int64_t* labels,
                                   int64_t lb, int64_t lt, void* out_lp0, void* out_lp1,
                                   int out_dtype, float* out_lse0, float* out_lse1, void* stream) {
    RowArgs a = {};
    a.x0 = x0; a.x1 = x1; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st;
    a.labels = labels; a.lb = lb; a.lt = lt;
    a.lp0 = out_lp0; a.lp1 = out_lp1; a.out_dtype = out_dtype; a.lse0 = out_lse0; a.lse1 = out_lse1;
    if (B * T == 0 && B >= 0 && T >= 0) return TRLX_OK;  // empty batch: nothing to launch
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(out_lp0 && (!x1 || out_lp1), TRLX_ERR_ARG, "NULL logprob output");
    TRLX_REQUIRE(out_dtype == TRLX_F32 || out_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "out dtype");
    return launch_rows<kFwd>(a, dtype, x1 ? 2 : 1, (hipStream_t)stream);
}

extern "C" int64_t trlx_ragged_order_bytes(int64_t B, int64_t T) { return ragged_order_bytes(B, T); }

extern "C" int trlx_lsm_gather_fwd_ragged(const void* x0, const void* x1, int dtype, int64_t B, int64_t T,
                                          int64_t V, int64_t sb, int64_t st, const int64_t* labels, int64_t lb,
                                          int64_t lt, const int64_t* lengths, void* order_ws, void* out_lp0,
                                          void* out_lp1, int out_dtype, void* stream) {
    RowArgs a = {};
    a.x0 = x0; a.x1 = x1; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st;
    a.labels = labels; a.lb = lb; a.lt = lt; a.lengths = lengths; a.order_ws = static_cast<int*>(order_ws);
    a.lp0 = out_lp0; a.lp1 = out_lp1; a.out_dtype = out_dtype;
    if (B * T == 0 && B >= 0 && T >= 0) return TRLX_OK;
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(out_lp0 && (!x1 || out_lp1), TRLX_ERR_ARG, "NULL logprob output");
    TRLX_REQUIRE(out_dtype == TRLX_F32 || out_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "out dtype");
    return launch_rows<kFwd>(a, dtype, x1 ? 2 : 1, (hipStream_t)stream);
}

static int fill_loss_tail(LossRolloutArgs* L, int64_t B, int64_t T, const double* stats, float vf_coef, float* loss,
                          float* loss_stats, void* workspace, const trlx_kl_ctl* kl);

extern "C" int trlx_lsm_gather_fwd_loss_tail(const void* x0, const void* x1, int dtype, int64_t B, int64_t T,
                                             int64_t V, int64_t sb, int64_t st, const int64_t* labels, int64_t lb,
                                             int64_t lt, const int64_t* lengths, void* order_ws, void* out_lp0,
                                             void* out_lp1, int out_dtype, int64_t tail_B, int64_t tail_T,
                                             const double* tail_stats, float vf_coef, float* loss, float* loss_stats,
                                             void* workspace, const trlx_kl_ctl* kl, void* stream) {
    RowArgs a = {};
    a.x0 = x0; a.x1 = x1; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st;
    a.labels = labels; a.lb = lb; a.lt = lt; a.lengths = lengths; a.order_ws = static_cast<int*>(order_ws);
    a.lp0 = out_lp0; a.lp1 = out_lp1; a.out_dtype = out_dtype;
    int rc = fill_loss_tail(&a.tail, tail_B, tail_T, tail_stats, vf_coef, loss, loss_stats, workspace, kl);
    if (rc) return rc;
    a.has_tail = 1;
    if (B * T == 0 && B >= 0 && T >= 0) return lead_standalone(a, (hipStream_t)stream, true, false);
    rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(out_lp0 && (!x1 || out_lp1), TRLX_ERR_ARG, "NULL logprob output");
    TRLX_REQUIRE(out_dtype == TRLX_F32 || out_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "out dtype");
    return launch_rows<kFwd>(a, dtype, x1 ? 2 : 1, (hipStream_t)stream);
}

extern "C" int trlx_lsm_gather_bwd(const void* x, int dtype, int64_t B, int64_t T, int64_t V,
                                   int64_t sb, int64_t st, const int64_t* labels, int64_t lb,
                                   int64_t lt, const float* lse, const void* grad, int grad_dtype,
                                   void* dx, int64_t dsb, int64_t dst, void* stream) {
    RowArgs a = {};
    a.x0 = x; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st; a.labels = labels; a.lb = lb; a.lt = lt;
    a.lse_in = lse; a.grad = grad; a.grad_dtype = grad_dtype; a.dx = dx; a.dsb = dsb; a.dst = dst;
    if (B * T == 0 && B >= 0 && T >= 0) return TRLX_OK;
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(lse && grad && dx, TRLX_ERR_ARG, "NULL lse/grad/dx");
    return launch_rows<kBwd>(a, dtype, 1, (hipStream_t)stream);
}

extern "C" int trlx_ppo_policy_fused(const void* x, int dtype, int64_t B, int64_t T, int64_t V,
                                     int64_t sb, int64_t st, const int64_t* labels, int64_t lb,
                                     int64_t lt, const void* old_lp, int old_dtype, const float* adv,
                                     const double* stats, int unbiased, const int64_t* mask,
                                     const double* msum, double msum_host, float cliprange,
                                     float* lp_out, void* dx, int64_t dsb, int64_t dst, void* stream) {
    RowArgs a = {};
    a.x0 = x; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st; a.labels = labels; a.lb = lb; a.lt = lt;
    a.old_lp = old_lp; a.old_dtype = old_dtype; a.adv = adv; a.stats = stats; a.unbiased = unbiased;
    a.mask = mask; a.msum = msum; a.msum_host = msum_host; a.cliprange = cliprange;
    a.lp_out = lp_out; a.dx = dx; a.dsb = dsb; a.dst = dst;
    if (B * T == 0 && B >= 0 && T >= 0) return TRLX_OK;
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(old_lp && adv && lp_out && dx, TRLX_ERR_ARG, "NULL old_lp/adv/lp_out/dx");
    TRLX_REQUIRE(msum || msum_host > 0, TRLX_ERR_ARG, "mask sum must be positive");
    return launch_rows<kPpo>(a, dtype, 1, (hipStream_t)stream);
}

extern "C" int64_t trlx_ppo_workspace_bytes(int64_t B, int64_t T) {
    return int64_t(carve_workspace(nullptr, B, T, nullptr));
}

// Split-beta outputs of the GAE launch (k_rollout_gae<true>); NULL = the unsplit launch.
struct SplitGae {
    float *adv_kl, *rew_kl, *rew_score;
    const double* prev_stats;
    float* prev_coef;
    int prev_unbiased;
    int mom_lag;          // ScoreCtlArgs::lag
    void* done_event;     // recorded by the launch's own dispatch (hipExtLaunchKernel), or NULL
};

static int fill_gae(GaeRolloutArgs& e, int64_t B, int64_t T, const float* lp, const float* ref_lp, const void* values,
                    int v_dtype, const float* scores, const int64_t* lengths, const int64_t* mask, float kl_coef,
                    const trlx_score_ctl* ctl, float gamma, float lam, float* rewards, float* adv_raw, void* ret,
                    int ret_dtype, double* stats, void* workspace, const SplitGae* sp) {
    TRLX_REQUIRE(B > 0 && T > 0 && B * T < (1LL << 31), TRLX_ERR_SHAPE, "bad rollout batch %lld x %lld",
                 (long long)B, (long long)T);
    TRLX_REQUIRE(lp && ref_lp && values && adv_raw && stats && workspace && (sp || (rewards && ret)), TRLX_ERR_ARG,
                 "NULL argument to trlx_ppo_rollout_gae");
    e = {};
    carve_workspace(workspace, B, T, &e.ws);
    e.B = int(B); e.T = int(T); e.lp = lp; e.ref_lp = ref_lp; e.values = values; e.v_dtype = v_dtype;
    e.scores = scores; e.lengths = lengths; e.mask = mask; e.neg_beta = -kl_coef; e.gamma = gamma;
    e.gl = float(double(gamma) * double(lam));  // python float product, then fp32 (torch scalar)
    e.rewards = rewards; e.adv = adv_raw; e.ret = ret; e.ret_dtype = ret_dtype; e.stats = stats;
    if (ctl) {
        TRLX_REQUIRE(scores && ctl->state_in && ctl->state_out, TRLX_ERR_ARG,
                     "score control needs scores, state_in and state_out");
        TRLX_REQUIRE(ctl->state_in != ctl->state_out, TRLX_ERR_ARG,
                     "trlx_ppo_rollout_gae_ctl: state_out must not alias state_in (every block reads it)");
        TRLX_REQUIRE(ctl->scale_mode >= TRLX_SCALE_NONE && ctl->scale_mode <= TRLX_SCALE_REF, TRLX_ERR_ARG,
                     "bad scale_mode %d", ctl->scale_mode);
        e.has_ctl = 1;
        e.ctl.state_in = ctl->state_in; e.ctl.state_out = ctl->state_out; e.ctl.global_mom = ctl->global_moments;
        e.ctl.scale_mode = ctl->scale_mode; e.ctl.clip = ctl->cliprange_reward;
        if (sp && sp->mom_lag) {
            TRLX_REQUIRE(ctl->scale_mode != TRLX_SCALE_RUNNING, TRLX_ERR_ARG,
                         "lagged score moments cannot scale by the running std (it needs this batch's moments)");
            e.ctl.lag = 1;
        }
    }
    if (sp) {
        TRLX_REQUIRE(sp->adv_kl && sp->rew_kl && sp->rew_score, TRLX_ERR_ARG, "NULL split-beta GAE output");
        TRLX_REQUIRE(!sp->prev_stats || sp->prev_coef, TRLX_ERR_ARG, "prev_stats needs prev_coef");
        e.adv_kl = sp->adv_kl; e.rew_kl = sp->rew_kl; e.rew_score = sp->rew_score;
        e.prev_stats = sp->prev_stats; e.prev_coef = sp->prev_coef; e.prev_unbiased = sp->prev_unbiased;
        e.host_beta = kl_coef;
    }
    return TRLX_OK;
}

static int rollout_gae_impl(int64_t B, int64_t T, const float* lp, const float* ref_lp, const void* values,
                            int v_dtype, const float* scores, const int64_t* lengths, const int64_t* mask,
                            float kl_coef, const trlx_score_ctl* ctl, float gamma, float lam, float* rewards,
                            float* adv_raw, void* ret, int ret_dtype, double* stats, void* workspace, void* stream,
                            const SplitGae* sp = nullptr) {
    GaeRolloutArgs e;
    const int rc = fill_gae(e, B, T, lp, ref_lp, values, v_dtype, scores, lengths, mask, kl_coef, ctl, gamma, lam,
                            rewards, adv_raw, ret, ret_dtype, stats, workspace, sp);
    if (rc) return rc;
    const unsigned nblk = unsigned((B + kRolloutsPerBlock - 1) / kRolloutsPerBlock);
    if (e.adv_kl && sp->done_event)  // the side stream's ordering point rides the dispatch (no marker packet)
        hipExtLaunchKernelGGL(k_rollout_gae<true>, dim3(nblk), dim3(kRolloutThreads), 0, (hipStream_t)stream, nullptr,
                              (hipEvent_t)sp->done_event, 0, e);
    else if (e.adv_kl)
        hipLaunchKernelGGL(k_rollout_gae<true>, dim3(nblk), dim3(kRolloutThreads), 0, (hipStream_t)stream, e);
    else
        hipLaunchKernelGGL(k_rollout_gae<false>, dim3(nblk), dim3(kRolloutThreads), 0, (hipStream_t)stream, e);
    return check_launch("k_rollout_gae");
}

extern "C" int trlx_ppo_rollout_gae(int64_t B, int64_t T, const float* lp, const float* ref_lp, const void* values,
                                    int v_dtype, const float* scores, const int64_t* lengths, const int64_t* mask,
                                    float kl_coef, float gamma, float lam, float* rewards, float* adv_raw, void* ret,
                                    int ret_dtype, double* stats, void* workspace, void* stream) {
    return rollout_gae_impl(B, T, lp, ref_lp, values, v_dtype, scores, lengths, mask, kl_coef, nullptr, gamma, lam,
                            rewards, adv_raw, ret, ret_dtype, stats, workspace, stream);
}

extern "C" int trlx_ppo_rollout_gae_ctl(int64_t B, int64_t T, const float* lp, const float* ref_lp,
                                        const void* values, int v_dtype, const float* scores,
                                        const int64_t* lengths, const int64_t* mask, const trlx_score_ctl* ctl,
                                        float gamma, float lam, float* rewards, float* adv_raw, void* ret,
                                        int ret_dtype, double* stats, void* workspace, void* stream) {
    TRLX_REQUIRE(ctl, TRLX_ERR_ARG, "NULL trlx_score_ctl");
    return rollout_gae_impl(B, T, lp, ref_lp, values, v_dtype, scores, lengths, mask, 0.0f, ctl, gamma, lam,
                            rewards, adv_raw, ret, ret_dtype, stats, workspace, stream);
}

extern "C" int trlx_ppo_rollout_gae_split(int64_t B, int64_t T, const float* lp, const float* ref_lp,
                                          const void* values, int v_dtype, const float* scores,
                                          const int64_t* lengths, const int64_t* mask, const trlx_score_ctl* ctl,
                                          float kl_coef, float gamma, float lam, float* adv0, float* adv_kl,
                                          float* rew_kl, float* rew_score, double* stats8, const double* prev_stats8,
                                          float* prev_coef, int prev_unbiased, int mom_lag, void* workspace,
                                          void* stream, void* done_event) {
    const SplitGae sp = {adv_kl, rew_kl, rew_score, prev_stats8, prev_coef, prev_unbiased, mom_lag, done_event};
    return rollout_gae_impl(B, T, lp, ref_lp, values, v_dtype, scores, lengths, mask, kl_coef, ctl, gamma, lam,
                            nullptr, adv0, nullptr, TRLX_F32, stats8, workspace, stream, &sp);
}

extern "C" int trlx_ppo_whiten_coef(const double* stats8, int unbiased, const double* ctl_state, float kl_coef,
                                    float* coef, void* stream) {
    TRLX_REQUIRE(stats8 && coef, TRLX_ERR_ARG, "NULL argument to trlx_ppo_whiten_coef");
    hipLaunchKernelGGL(k_whiten_coef, dim3(1), dim3(kWave), 0, (hipStream_t)stream, stats8, unbiased, ctl_state,
                       kl_coef, coef);
    return check_launch("k_whiten_coef");
}

extern "C" int trlx_ppo_experience_fused(const void* logits, const void* ref_logits, int dtype, int64_t B,
                                         int64_t T, int64_t V, int64_t sb, int64_t st, const int64_t* labels,
                                         int64_t lb, int64_t lt, const void* values, int v_dtype,
                                         const float* scores, const int64_t* lengths, const int64_t* mask,
                                         float kl_coef, float gamma, float lam, float* lp, float* ref_lp,
                                         float* rewards, float* adv_raw, void* ret, int ret_dtype,
                                         double* stats, void* workspace, void* stream) {
    TRLX_REQUIRE(ref_logits && workspace, TRLX_ERR_ARG, "NULL reference logits / workspace");
    Workspace ws;
    carve_workspace(workspace, B, T, &ws);
    int rc = trlx_lsm_gather_fwd_ragged(logits, ref_logits, dtype, B, T, V, sb, st, labels, lb, lt, lengths, ws.order,
                                        lp, ref_lp, TRLX_F32, stream);
    if (rc) return rc;
    return trlx_ppo_rollout_gae(B, T, lp, ref_lp, values, v_dtype, scores, lengths, mask, kl_coef, gamma, lam,
                                rewards, adv_raw, ret, ret_dtype, stats, workspace, stream);
}

extern "C" int trlx_ppo_loss_rows(const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb,
                                  int64_t st, const int64_t* labels, int64_t lb, int64_t lt, const void* old_lp,
                                  int old_dtype, const float* adv_raw, const double* stats, int unbiased,
                                  const int64_t* mask, const void* values, int v_dtype, const void* old_values,
                                  int ov_dtype, const void* returns, int r_dtype, float cliprange,
                                  float cliprange_value, float vf_coef, float* lp_out, void* dx, int64_t dsb,
                                  int64_t dst, float* dvalues, void* workspace, void* stream) {
    RowArgs a = {};
    a.x0 = logits; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st; a.labels = labels; a.lb = lb; a.lt = lt;
    a.old_lp = old_lp; a.old_dtype = old_dtype; a.adv = adv_raw; a.stats = stats; a.unbiased = unbiased;
    a.mask = mask; a.msum = stats ? stats + 3 : nullptr; a.msum_host = double(B * T); a.cliprange = cliprange;
    a.lp_out = lp_out; a.dx = dx; a.dsb = dsb; a.dst = dst;
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(B > 0 && T > 0, TRLX_ERR_SHAPE, "empty rollout batch");
    TRLX_REQUIRE(old_lp && adv_raw && stats && values && old_values && returns && lp_out && dx && dvalues && workspace,
                 TRLX_ERR_ARG, "NULL argument to trlx_ppo_loss_rows");
    Workspace ws;
    carve_workspace(workspace, B, T, &ws);
    a.tokrec = ws.tokrec;
    a.ltok.values = values; a.ltok.v_dtype = v_dtype; a.ltok.old_values = old_values; a.ltok.ov_dtype = ov_dtype;
    a.ltok.returns = returns; a.ltok.r_dtype = r_dtype; a.ltok.cv = cliprange_value; a.ltok.vf_coef = vf_coef;
    a.ltok.dv = dvalues;
    return launch_rows<kPpo>(a, dtype, 1, (hipStream_t)stream);
}

extern "C" int trlx_ppo_loss_rows_split(const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb,
                                        int64_t st, const int64_t* labels, int64_t lb, int64_t lt, const void* old_lp,
                                        int old_dtype, const float* adv0, const float* adv_kl, const float* rew_kl,
                                        const float* rew_score, const float* coef, const double* msum,
                                        const int64_t* mask, const void* values, int v_dtype, const void* old_values,
                                        int ov_dtype, float* rewards, void* returns, int r_dtype, float cliprange,
                                        float cliprange_value, float vf_coef, float* lp_out, void* dx, int64_t dsb,
                                        int64_t dst, float* dvalues, void* workspace, void* stream) {
    RowArgs a = {};
    a.x0 = logits; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st; a.labels = labels; a.lb = lb; a.lt = lt;
    a.old_lp = old_lp; a.old_dtype = old_dtype; a.adv = adv0; a.adv_kl = adv_kl; a.rew_kl = rew_kl;
    a.rew_score = rew_score; a.coef = coef; a.rewards_out = rewards;
    a.mask = mask; a.msum = msum; a.msum_host = double(B * T); a.cliprange = cliprange;
    a.lp_out = lp_out; a.dx = dx; a.dsb = dsb; a.dst = dst;
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(B > 0 && T > 0, TRLX_ERR_SHAPE, "empty rollout batch");
    TRLX_REQUIRE(old_lp && adv0 && adv_kl && rew_kl && rew_score && coef && rewards && values && old_values &&
                 returns && lp_out && dx && dvalues && workspace, TRLX_ERR_ARG,
                 "NULL argument to trlx_ppo_loss_rows_split");
    TRLX_REQUIRE(r_dtype == TRLX_F32 || r_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "returns dtype %d", r_dtype);
    Workspace ws;
    carve_workspace(workspace, B, T, &ws);
    a.tokrec = ws.tokrec;
    a.ltok.values = values; a.ltok.v_dtype = v_dtype; a.ltok.old_values = old_values; a.ltok.ov_dtype = ov_dtype;
    a.ltok.returns = returns; a.ltok.r_dtype = r_dtype; a.ltok.cv = cliprange_value; a.ltok.vf_coef = vf_coef;
    a.ltok.dv = dvalues;
    return launch_rows<kPpo>(a, dtype, 1, (hipStream_t)stream);
}

extern "C" int trlx_ppo_loss_rows_split_gae(
    const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb, int64_t st, const int64_t* labels,
    int64_t lb, int64_t lt, const void* old_lp, int old_dtype, const float* adv0, const float* adv_kl,
    const float* rew_kl, const float* rew_score, const double* stats8, int unbiased, const double* ctl_state,
    float kl_coef, float* coef, const double* msum, const int64_t* mask, const void* values, int v_dtype,
    const void* old_values, int ov_dtype, float* rewards, void* returns, int r_dtype, float cliprange,
    float cliprange_value, float vf_coef, float* lp_out, void* dx, int64_t dsb, int64_t dst, float* dvalues,
    void* workspace, const trlx_gae_split_args* gae, void* stream, void* done_event) {
    RowArgs a = {};
    a.x0 = logits; a.B = B; a.T = T; a.V = V; a.sb = sb; a.st = st; a.labels = labels; a.lb = lb; a.lt = lt;
    a.old_lp = old_lp; a.old_dtype = old_dtype; a.adv = adv0; a.adv_kl = adv_kl; a.rew_kl = rew_kl;
    a.rew_score = rew_score; a.rewards_out = rewards;
    a.wstats = stats8; a.wunbiased = unbiased; a.wctl = ctl_state; a.wbeta = kl_coef; a.coef_out = coef;
    a.mask = mask; a.msum = msum; a.msum_host = double(B * T); a.cliprange = cliprange;
    a.lp_out = lp_out; a.dx = dx; a.dsb = dsb; a.dst = dst;
    a.done_event = done_event;
    int rc = check_rows(a, dtype);
    if (rc) return rc;
    TRLX_REQUIRE(B > 0 && T > 0, TRLX_ERR_SHAPE, "empty rollout batch");
    TRLX_REQUIRE(old_lp && adv0 && adv_kl && rew_kl && rew_score && stats8 && rewards && values && old_values &&
                 returns && lp_out && dx && dvalues && workspace, TRLX_ERR_ARG,
                 "NULL argument to trlx_ppo_loss_rows_split_gae");
    TRLX_REQUIRE(r_dtype == TRLX_F32 || r_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "returns dtype %d", r_dtype);
    Workspace ws;
    carve_workspace(workspace, B, T, &ws);
    a.tokrec = ws.tokrec;
    a.ltok.values = values; a.ltok.v_dtype = v_dtype; a.ltok.old_values = old_values; a.ltok.ov_dtype = ov_dtype;
    a.ltok.returns = returns; a.ltok.r_dtype = r_dtype; a.ltok.cv = cliprange_value; a.ltok.vf_coef = vf_coef;
    a.ltok.dv = dvalues;
    if (gae) {
        // the GAE's tickets / block records and the rows' token records share a workspace
        // only when it is carved for the same batch shape
        TRLX_REQUIRE(gae->workspace != workspace || (gae->B == B && gae->T == T), TRLX_ERR_ARG,
                     "folded GAE of a %lld x %lld batch cannot share the %lld x %lld loss workspace",
                     (long long)gae->B, (long long)gae->T, (long long)B, (long long)T);
        TRLX_REQUIRE(gae->stats8 != stats8 && gae->adv0 != adv0 && gae->adv_kl != adv_kl, TRLX_ERR_ARG,
                     "the folded GAE must write the other split buffer set (it runs beside these rows)");
        const SplitGae sp = {gae->adv_kl, gae->rew_kl, gae->rew_score, nullptr, nullptr, 0, gae->mom_lag, nullptr};
        rc = fill_gae(a.gae, gae->B, gae->T, gae->lp, gae->ref_lp, gae->values, gae->v_dtype, gae->scores,
                      gae->lengths, gae->mask, gae->kl_coef, gae->ctl, gae->gamma, gae->lam, nullptr, gae->adv0,
                      nullptr, TRLX_F32, gae->stats8, gae->workspace, &sp);
        if (rc) return rc;
        TRLX_REQUIRE(!gae->ctl || (ctl_state != gae->ctl->state_out), TRLX_ERR_ARG,
                     "the rows read beta from the state the folded GAE writes (pass its state_in)");
        a.has_gae = 1;
    }
    return launch_rows<kPpo>(a, dtype, 1, (hipStream_t)stream);
}

static int fill_loss_tail(LossRolloutArgs* L, int64_t B, int64_t T, const double* stats, float vf_coef, float* loss,
                          float* loss_stats, void* workspace, const trlx_kl_ctl* kl) {
    TRLX_REQUIRE(B > 0 && T > 0, TRLX_ERR_SHAPE, "empty rollout batch");
    TRLX_REQUIRE(loss && loss_stats && workspace, TRLX_ERR_ARG, "NULL argument to the PPO loss tail");
    *L = {};
    carve_workspace(workspace, B, T, &L->ws);
    L->B = int(B); L->T = int(T); L->msum = stats ? stats + 3 : nullptr; L->vf_coef = vf_coef; L->loss = loss;
    L->stats = loss_stats;
    if (kl) {
        TRLX_REQUIRE(kl->state, TRLX_ERR_ARG, "trlx_kl_ctl.state is NULL");
        TRLX_REQUIRE(!kl->adaptive || (kl->target != 0.0 && kl->horizon != 0.0), TRLX_ERR_ARG,
                     "adaptive KL control needs target and horizon");
        L->kl.state = kl->state; L->kl.adaptive = kl->adaptive; L->kl.target = kl->target;
        L->kl.horizon = kl->horizon; L->kl.n_steps = double(kl->n_steps);
    }
    return TRLX_OK;
}

static int rollout_loss_impl(int64_t B, int64_t T, const double* stats, float vf_coef, float* loss,
                             float* loss_stats, void* workspace, const trlx_kl_ctl* kl, void* stream) {
    LossRolloutArgs L;
    const int rc = fill_loss_tail(&L, B, T, stats, vf_coef, loss, loss_stats, workspace, kl);
    if (rc) return rc;
    const unsigned nblk = unsigned((B + kRolloutsPerBlock - 1) / kRolloutsPerBlock);
    hipLaunchKernelGGL(k_rollout_loss, dim3(nblk), dim3(kRolloutThreads), 0, (hipStream_t)stream, L);
    return check_launch("k_rollout_loss");
}

extern "C" int trlx_ppo_rollout_loss(int64_t B, int64_t T, const double* stats, float vf_coef, float* loss,
                                     float* loss_stats, void* workspace, void* stream) {
    return rollout_loss_impl(B, T, stats, vf_coef, loss, loss_stats, workspace, nullptr, stream);
}

extern "C" int trlx_ppo_rollout_loss_ctl(int64_t B, int64_t T, const double* stats, float vf_coef, float* loss,
                                         float* loss_stats, void* workspace, const trlx_kl_ctl* kl, void* stream) {
    TRLX_REQUIRE(kl, TRLX_ERR_ARG, "NULL trlx_kl_ctl");
    return rollout_loss_impl(B, T, stats, vf_coef, loss, loss_stats, workspace, kl, stream);
}

extern "C" int trlx_ppo_loss_fused(const void* logits, int dtype, int64_t B, int64_t T, int64_t V, int64_t sb,
                                   int64_t st, const int64_t* labels, int64_t lb, int64_t lt, const void* old_lp,
                                   int old_dtype, const float* adv_raw, const double* stats, int unbiased,
                                   const int64_t* mask, const void* values, int v_dtype, const void* old_values,
                                   int ov_dtype, const void* returns, int r_dtype, float cliprange,
                                   float cliprange_value, float vf_coef, float* lp_out, void* dx, int64_t dsb,
                                   int64_t dst, float* dvalues, float* loss, float* loss_stats, void* workspace,
                                   void* stream) {
    int rc = trlx_ppo_loss_rows(logits, dtype, B, T, V, sb, st, labels, lb, lt, old_lp, old_dtype, adv_raw, stats,
                                unbiased, mask, values, v_dtype, old_values, ov_dtype, returns, r_dtype, cliprange,
                                cliprange_value, vf_coef, lp_out, dx, dsb, dst, dvalues, workspace, stream);
    if (rc) return rc;
    return trlx_ppo_rollout_loss(B, T, stats, vf_coef, loss, loss_stats, workspace, stream);
}

extern "C" int trlx_set_tuning(const char* key, int64_t value) {
    const std::string k = key ? key : "";
    if (k == "row_variant") g_row_variant = int(value);
    else if (k == "resident_lb512") g_resident_lb512 = int(value);
    else if (k == "resident_threads") {
        TRLX_REQUIRE(value == 0 || (value % kWave == 0 && value <= kMaxThreads), TRLX_ERR_ARG,
                     "resident_threads must be a multiple of 64 <= %d", kMaxThreads);
        g_resident_threads = int(value);
    } else if (k == "stream_threads") {
        TRLX_REQUIRE(value == 0 || (value % kWave == 0 && value <= kStreamMaxThreads), TRLX_ERR_ARG,
                     "stream_threads must be a multiple of 64 <= %d", kStreamMaxThreads);
        g_stream_threads = int(value);
    } else if (k == "ilql_split") {
        TRLX_REQUIRE(value >= 0 && value <= 3, TRLX_ERR_ARG, "ilql_split: 0 (20+5), 1 (22+3), 2 (21+4), 3 (19+6)");
        g_ilql_split = int(value);
    } else if (k == "split_lds") {
        TRLX_REQUIRE(value >= 0 && value <= 2, TRLX_ERR_ARG, "split_lds: 0..2");
        g_split_lds = int(value);
    } else if (k == "store_policy") {
        TRLX_REQUIRE(value >= 0 && value <= 5, TRLX_ERR_ARG, "store_policy: 0..5");
        g_store_pol = int(value);
    } else if (k == "split_mid") {
        TRLX_REQUIRE(value >= 0 && value <= 3, TRLX_ERR_ARG, "split_mid: 0..3");
        g_split_mid = int(value);
    } else if (k == "order_launch") {
        TRLX_REQUIRE(value >= 0 && value <= 2, TRLX_ERR_ARG, "order_launch: 0 auto, 1 one launch, 2 two launches");
        g_order_launch = int(value);
    } else if (k == "ragged_order") {
        TRLX_REQUIRE(value == 0 || value == 1, TRLX_ERR_ARG, "ragged_order: 0 (valid rows first) or 1 (natural)");
        g_ragged_order = int(value);
    } else if (k == "row_order") {
        TRLX_REQUIRE(value == 0 || value == 1, TRLX_ERR_ARG, "row_order: 0 or 1");
        g_row_order = int(value);
    } else if (k == "stream_unroll") {
        TRLX_REQUIRE(value == 0 || value == 2 || value == 4 || value == 8, TRLX_ERR_ARG, "stream_unroll: 2, 4 or 8");
        g_stream_unroll = int(value);
    } else {
        bool handled = false;
        const int rc = lmloss_set_tuning(key, value, &handled);
        if (handled) return rc;
        set_error("unknown tuning key '%s'", k.c_str());
        return TRLX_ERR_ARG;
    }
    return TRLX_OK;
}
