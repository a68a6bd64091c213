// Fused lm_head + log-softmax-gather with its BACKWARD, for the PPO loss side (SURVEY §8f
// rank 2): the policy update's [N, V] logits and dlogits never reach HBM.
//
//   reference (accelerate_ppo_model.py:96-118):  logits = lm_head(h)            ppo_models.py:640 / :274
//                                                lp = logprobs_from_logits(logits, y)   modeling.py:37-41
//                                                loss = PPOConfig.loss(lp, ...)          ppo_models.py:141-199
//                                                autograd -> dlogits [N, V] -> dh = dlogits·W, dW = dlogitsᵀ·h
//
// With p = softmax(h·Wᵀ) and g_t = d loss / d lp_t the gradients are
//   dh_t = g_t · (W[y_t] − Σ_v p_tv · W_v)          dW_v = Σ_t g_t · (1[y_t = v] − p_tv) · h_t
// so the loss side runs as (FLOPs in units of one N·V·H multiply-add pass):
//   k_lmloss_fwd      per token tile, the online softmax over a split of the vocab and the
//                     "expected embedding" O = Σ_v exp(x_tv − m) · W_v next to it (flash-style:
//                     S = W_tile·hᵀ and O += W_tileᵀ·P on MFMA, 2 passes): partial (m, l, O)
//                     per (token, vocab split), the label logit
//   k_lmloss_combine  per token: merge the splits -> lse, lp, E = O / l; g_t from the PPO loss
//                     (ppo_token.h, the loss rows' own per-token arithmetic) or from a caller's
//                     d loss / d lp; dh_t = g_t (W[y_t] − E_t); the per-token loss record
//   k_lmloss_dw       per vocab tile, every token tile: S = h_tile·W_tileᵀ recomputed, the
//                     dlogits tile g·(onehot − exp(S − lse)) formed in registers (bf16) and
//                     dW_tile += dSᵀ·h_tile on MFMA (2 passes), fixed order over token tiles
// 4 passes in all (the unfused path: logits GEMM, rows, dh GEMM, dW GEMM = 3 passes plus ~4·N·V
// bytes of logits / dlogits traffic).  Deterministic: no atomics, fixed reduction orders.
//
// MFMA v_mfma_f32_32x32x16_bf16 throughout.  A workgroup is 4 waves = 2 pairs x 2 hidden
// halves: each pair owns 32 tokens (forward) or 32 vocab rows (dW); the two waves of a pair
// each hold HALF of the hidden dimension (their h / W fragments in registers and their half of
// O / dW as accumulators: 96 + 192 registers at H = 768) and add their partial S tiles
// through LDS, so the S product reads each staged operand once per pair and both products use
// the 32 x 32 shape (half the LDS operand bytes per FLOP of 16 x 16).  The accumulator of S
// (vocab or token on the MFMA rows) is the B / A operand of the second product with no lane
// movement (cdna_hip_programming.md §3 'An accumulator tile as the next MFMA's operand'); the
// streamed tile is read by rows (ds_read_b128) for S and by columns (ds_read_b64_tr_b16) for
// the second product from ONE swizzled LDS image.
#define TRLX_ROW_TAILS_NO_KERNELS
#include "ppo_token.h"

namespace trlx {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int kLLRows = 32;            // rows of a staged tile: vocab rows (forward) / tokens (dW)
constexpr int kLLThreads = 256;        // 2 pairs x 2 hidden halves
constexpr int kLLTokTile = 64;         // tokens per forward workgroup (2 pairs x 32)
constexpr int kLLVocTile = 64;         // vocab rows per dW workgroup
constexpr int kLLMaxSplits = 8;        // vocab splits of the forward (workspace sizing)
constexpr float kLLOverflow = 60.0f;   // logit - offset bound of the fixed-offset softmax (e^60)
constexpr int kLLXchg = 4 * 4096;      // partial-S exchange: 16 fp32 per lane per wave

enum LmLossMode { kLLPpo = 0, kLLFwd = 1, kLLBwd = 2 };

struct LmLossArgs {
    const uint16_t* h;   // [N, ldh] bf16 hidden states
    const uint16_t* w;   // [V, ldw] bf16 lm_head weight (nn.Linear layout)
    int64_t ldh, ldw;
    int N, H, V;
    const int64_t* labels;  // [N] (token rows)
    int64_t lb;             // label stride
    // compaction: rows[m] = row of compact token m < *nrows (mask != 0), ~row of the masked
    // ones after them (k_mask_order); NULL = every token, row m
    const int* rows;
    const int* nrows;
    int nsplit;
    float* opart;    // [nsplit][N][H] partial O (compact token index)
    float2* mlpart;  // [nsplit][N] partial (m, l)
    float* xlab;     // [N] label logit (compact)
    float* nlse;     // [N] -lse·log2e (compact; read by the dW kernel)
    float* gbuf;     // [N] d loss / d lp (compact)
    int* ybuf;       // [N] label (compact)
    float* ebuf;     // kLLFwd: E = O / l written here; kLLBwd: read ([N, H], token rows)
    float* lse_io;   // kLLFwd: lse out; kLLBwd: lse in (token rows); may be NULL in kLLPpo
    void* lp;        // lp out (token rows; kLLPpo: fp32 lp_out)
    int lp_dtype;
    const void* gin; // kLLBwd: d loss / d lp (token rows)
    int gin_dtype;
    void* dh;        // [N, lddh] d hidden (token rows)
    int64_t lddh;
    int dh_dtype;
    void* dw;        // [V, lddw] d weight of dw_dtype (or [tsplit][V][H] fp32 partials)
    int64_t lddw;
    int dw_dtype;
    int tsplit;
    int mode;
    // ---- per-token PPO fields (the names ppo_token.h reads; see RowArgs in vocab_rows.hip)
    const void* old_lp;
    int old_dtype;
    const float* adv;
    const double* stats;
    int unbiased;
    const int64_t* mask;
    const double* msum;
    double msum_host;
    float cliprange;
    float* lp_out;
    float* tokrec;
    LossTokenArgs ltok;
    const float* coef;
    const float* adv_kl;
    const float* rew_kl;
    const float* rew_score;
    float* rewards_out;
    const double* wstats;
    int wunbiased;
    const double* wctl;
    float wbeta;
    float* coef_out;
};

// ------------------------------------------------------------------ staged tile image
// A [32 rows][H] bf16 tile as H/128 segments of [32 rows][256 B]; 16-B chunk c of a row sits at
// chunk c ^ key(row) of its segment row (cdna_hip_programming.md T10, image (b)): the row reads
// of the 32x32x16 operand (32 rows x one 16-B chunk per half-wave) and the transposed reads
// (4 rows x 16 columns per 16-lane group) are both conflict-free.
__device__ __forceinline__ int ll_key(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int ll_off(int r, int d) {
    return (d >> 7) * 8192 + r * 256 + ((((d >> 3) & 15) ^ ll_key(r)) << 4) + ((d & 7) << 1);
}

// One 1-KB LDS-DMA piece of a tile: piece i = segment i >> 3, rows 4(i & 7) .. +3; lane l
// lands at slot (row 4(i&7) + l/16, chunk l&15) and fetches the logical chunk (l&15) ^ key.
// `src_row` = the global row pointer of the lane's tile row.
__device__ __forceinline__ void ll_piece(char* slot, int i, const uint16_t* src_row, int lane) {
    const int r = 4 * (i & 7) + (lane >> 4);
    const int c = (lane & 15) ^ ll_key(r);
    __builtin_amdgcn_global_load_lds(src_row + (i >> 3) * 128 + c * 8,
                                     (__attribute__((address_space(3))) void*)(slot + i * 1024), 16, 0, 0);
}

// Row read of the 32x32x16 operand: lane l -> tile row l&31, 8 elements from column d0 + 8·(l>>5).
__device__ __forceinline__ bf16x8_t ll_row_frag(const char* slot, int lane, int d0) {
    return *reinterpret_cast<const bf16x8_t*>(slot + ll_off(lane & 31, d0 + 8 * (lane >> 5)));
}

// Transposed read of the 32x32x16 operand whose k runs over 16 tile rows in the order of an
// S accumulator used as the other operand (k-step s: element j of lane half hi is tile row
// 16s + 8(j>>2) + 4hi + (j&3)), column dcol0 + (l & 31): two ds_read_b64_tr_b16.
__device__ __forceinline__ bf16x8_t ll_tr_frag(const char* slot, int lane, int s, int dcol0) {
    const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
    const int r0 = 16 * s + 4 * (lane >> 5) + q;
    const int d = dcol0 + 16 * (g & 1) + 4 * p;
    typedef __attribute__((address_space(3))) s16x4_t lds_s4;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(slot + ll_off(r0, d)));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(slot + ll_off(r0 + 8, d)));
    const s16x8_t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ bf16x8_t pack8(const float* p) {
    bf16x8_t r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)p[j];
    return r;
}

// The two waves of a pair add their partial S tiles (each over its hidden half) through LDS:
// every lane ends with the full sum of its 16 elements (fp32 addition commutes, so both waves
// hold the same bits).  Barrier inside: every wave of the workgroup must call it.
__device__ __forceinline__ void ll_pair_sum(f32x16_t& s, char* xbuf, int wave, int lane) {
    f32x4_t* mine = reinterpret_cast<f32x4_t*>(xbuf + wave * 4096);
#pragma unroll
    for (int q = 0; q < 4; ++q) mine[q * 64 + lane] = f32x4_t{s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]};
    __syncthreads();
    const f32x4_t* oth = reinterpret_cast<const f32x4_t*>(xbuf + (wave ^ 1) * 4096);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f32x4_t o = oth[q * 64 + lane];
        s[4 * q] += o.x;
        s[4 * q + 1] += o.y;
        s[4 * q + 2] += o.z;
        s[4 * q + 3] += o.w;
    }
}

// ------------------------------------------------------------------ forward (flash-O)
// Workgroup = 64 tokens x one vocab split; wave (pair pr, half hh).  Per 32-row vocab tile:
//   S^T[v][t] = Σ_d W[v][d]·h[t][d]   (24 MFMAs over the wave's half, pair sum through LDS)
//   P = exp(S - offset) per token (lanes t and t^32 hold its 32 values), Σ P, label logit
//   O^T[d][t] += Σ_v W[v][d]·P[t][v] (12 d-blocks x 2 k-steps: W read transposed, P = the S
//   accumulator converted to bf16 as the B operand): each lane's O registers are ONE token's.
template <int KH>
__global__ __launch_bounds__(kLLThreads, 1) void k_lmloss_fwd(LmLossArgs a) {
    constexpr int HW = 16 * KH, H = 2 * HW, OB = HW / 32, NI = H / 64;
    constexpr int kStage = kLLRows * H * 2;
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage + kLLXchg];
    char* xbuf = smem + 2 * kStage;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, pr = wave >> 1, hh = wave & 1;
    const int hi = lane >> 5, c32 = lane & 31;
    const int nv = a.rows ? *a.nrows : a.N;
    const int split = int(blockIdx.x) % a.nsplit, mt = int(blockIdx.x) / a.nsplit;
    const int m0 = mt * kLLTokTile;
    if (m0 >= nv) return;  // past the compacted tokens (the grid's last blocks)
    const int tm = m0 + pr * 32 + c32;
    const bool valid = tm < nv;
    const int tc = valid ? tm : nv - 1;
    const int row = a.rows ? a.rows[tc] : tc;
    const int64_t y = valid ? a.labels[int64_t(row) * a.lb] : -1;
    bf16x8_t hf[KH];  // B operand of S^T: lane -> token c32, hidden hh·HW + 16ks + 8hi + j
    {
        const uint16_t* hp = a.h + int64_t(row) * a.ldh + hh * HW + 8 * hi;
#pragma unroll
        for (int ks = 0; ks < KH; ++ks) hf[ks] = *reinterpret_cast<const bf16x8_t*>(hp + 16 * ks);
    }
    const int nvt = (a.V + kLLRows - 1) / kLLRows;
    const int t0 = int(int64_t(split) * nvt / a.nsplit), t1 = int(int64_t(split + 1) * nvt / a.nsplit);
    auto issue = [&](int t, char* slot) {
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int i = wave + 4 * k;
            const int vr = min(t * kLLRows + 4 * (i & 7) + (lane >> 4), a.V - 1);
            ll_piece(slot, i, a.w + int64_t(vr) * a.ldw, lane);
        }
    };
    // The exponent offset of a token is FIXED for the whole split: the first tile's max (no
    // online rescale of O — a rescale of the 192 accumulators in a branch made the compiler
    // spill them, and a max that moves by < kLLOverflow leaves every term < e^60, in fp32 and
    // bf16 range).  If some token's logits exceed its offset by more than that, the workgroup
    // runs the split again with offset = the true max (never on realistic logits).
    f32x16_t O[OB];
    float mfix = -INFINITY, mtrue = -INFINITY, lrun = 0.0f;
    for (int pass = 0; pass < 2; ++pass) {
#pragma unroll
        for (int b = 0; b < OB; ++b) O[b] = f32x16_t{};
        lrun = 0.0f;
        bool bad = false;
        if (t0 < t1) issue(t0, smem);
        for (int t = t0; t < t1; ++t) {
            char* slot = smem + ((t - t0) & 1) * kStage;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's pieces of tile t
            __builtin_amdgcn_s_barrier();  // ... every wave's; and every wave is done with tile t-1
            if (t + 1 < t1) issue(t + 1, smem + ((t + 1 - t0) & 1) * kStage);
            f32x16_t s = f32x16_t{};
#pragma unroll
            for (int ks = 0; ks < KH; ++ks)
                s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ll_row_frag(slot, lane, hh * HW + 16 * ks), hf[ks], s, 0, 0,
                                                            0);
            ll_pair_sum(s, xbuf, wave, lane);
            // s[r] = logit(token c32, vocab t·32 + (r&3) + 8(r>>2) + 4hi)
            const int vb = t * kLLRows + 4 * hi;
            float mx = -INFINITY;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                if (vb + (r & 3) + 8 * (r >> 2) >= a.V) s[r] = -INFINITY;
                mx = fmaxf(mx, s[r]);
            }
            const int64_t dy = y - int64_t(t) * kLLRows;
            if (pass == 0 && hh == 0 && valid && dy >= 0 && dy < kLLRows && int((dy >> 2) & 1) == hi) {
                const int rr = int((dy & 3) + 4 * (dy >> 3));
                float xl = s[0];
#pragma unroll
                for (int r = 1; r < 16; ++r) xl = r == rr ? s[r] : xl;
                a.xlab[tm] = xl;
            }
            mx = fmaxf(mx, __shfl_xor(mx, 32));
            mtrue = fmaxf(mtrue, mx);
            if (pass == 0 && t == t0) mfix = mx;
            bad = bad || mx > mfix + kLLOverflow;
            const float nm = -mfix * kLog2e;
            float p[16];
            float ls = 0.0f;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                p[r] = exp2_fast(fmaf(s[r], kLog2e, nm));
                ls += p[r];
            }
            lrun += ls;
            const bf16x8_t pb0 = pack8(p), pb1 = pack8(p + 8);
#pragma unroll
            for (int b = 0; b < OB; ++b) {
                const int dc = hh * HW + 32 * b;
                O[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ll_tr_frag(slot, lane, 0, dc), pb0, O[b], 0, 0, 0);
                O[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ll_tr_frag(slot, lane, 1, dc), pb1, O[b], 0, 0, 0);
            }
        }
        if (!__syncthreads_or(bad)) break;
        mfix = mtrue;  // every tile's max is now <= the offset
    }
    const float mrun = mfix;
    const float ltok = lrun + __shfl_xor(lrun, 32);
    if (valid) {
        // O[b][r] = O(token c32, hidden hh·HW + 32b + (r&3) + 8(r>>2) + 4hi)
        float* op = a.opart + (int64_t(split) * a.N + tm) * a.H + hh * HW + 4 * hi;
#pragma unroll
        for (int b = 0; b < OB; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<f32x4_t*>(op + 32 * b + 8 * q) =
                    f32x4_t{O[b][4 * q], O[b][4 * q + 1], O[b][4 * q + 2], O[b][4 * q + 3]};
        if (hh == 0 && hi == 0) a.mlpart[int64_t(split) * a.N + tm] = make_float2(mrun, ltok);
    }
}

// ------------------------------------------------------------------ combine
// One workgroup per compact token m: merge the vocab splits (fixed order), lse, lp, g, dh.
template <int MODE>
__global__ __launch_bounds__(256) void k_lmloss_combine(LmLossArgs a) {
    const int m = blockIdx.x, tid = threadIdx.x;
    __shared__ float s_sc[kLLMaxSplits];
    __shared__ float s_tok[4];
    int row = m;
    bool pad = false;
    if (a.rows) {
        const int r = a.rows[m];
        pad = m >= *a.nrows;
        row = pad ? ~r : r;
    }
    const int H4 = a.H >> 2;
    if (pad) {  // a masked token (mask == 0): zero gradient, no logits needed (masked_row)
        if (MODE == kLLPpo && tid == 0) {
            float vin[3];
            const PpoScalars p = ppo_scalars(a, row, vin, true);
            PolicyTerms pt;
            ppo_policy_dlp(0.0f, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
            a.lp_out[row] = 0.0f;
            token_record(a, row, pt, p, vin);
            if (a.coef || a.wstats) split_outputs(a, row, p);
        }
        for (int d4 = tid; d4 < H4; d4 += blockDim.x) {
            if (a.dh_dtype == TRLX_BF16)
                reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.dh) + int64_t(row) * a.lddh)[d4] = make_uint2(0u, 0u);
            else
                reinterpret_cast<f32x4_t*>(static_cast<float*>(a.dh) + int64_t(row) * a.lddh)[d4] = f32x4_t{};
        }
        return;
    }
    const int64_t y = a.labels[int64_t(row) * a.lb];
    const bool yok = y >= 0 && y < a.V;
    float lse = 0.0f, L = 1.0f;
    if (MODE != kLLBwd) {
        float M = -INFINITY;
        for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.mlpart[int64_t(s) * a.N + m].x);
        L = 0.0f;
        for (int s = 0; s < a.nsplit; ++s) {
            const float2 p = a.mlpart[int64_t(s) * a.N + m];
            const float sc = p.x == -INFINITY ? 0.0f : exp2_fast((p.x - M) * kLog2e);
            L += p.y * sc;
            if (tid == s) s_sc[s] = sc;
        }
        const float lsum = logf(L);
        lse = M + lsum;
        if (tid == 0) {
            const float lp = yok ? (a.xlab[m] - M) - lsum : NAN;  // the reference's order, as in the rows
            float g = 0.0f;
            if (MODE == kLLPpo) {
                float vin[3];
                const PpoScalars p = ppo_scalars(a, row, vin, true);
                PolicyTerms pt;
                g = ppo_policy_dlp(lp, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
                const bool masked = p.m == 0.0f;
                a.lp_out[row] = masked ? 0.0f : lp;
                if (masked) ppo_policy_dlp(0.0f, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
                token_record(a, row, pt, p, vin);
                if (a.coef || a.wstats) split_outputs(a, row, p);
                a.gbuf[m] = g;
            } else {  // kLLFwd
                st_any(a.lp, a.lp_dtype, row, lp);
                if (a.lse_io) a.lse_io[row] = lse;
            }
            a.nlse[m] = -lse * kLog2e;
            a.ybuf[m] = yok ? int(y) : -1;
            s_tok[0] = g;
        }
    } else {  // kLLBwd: lse from the forward, g = the caller's d loss / d lp
        if (tid == 0) {
            lse = a.lse_io[row];
            const float g = ld_any(a.gin, a.gin_dtype, row);
            a.gbuf[m] = g;
            a.nlse[m] = -lse * kLog2e;
            a.ybuf[m] = yok ? int(y) : -1;
            s_tok[0] = g;
        }
    }
    __syncthreads();
    const float g = s_tok[0];
    const float invL = 1.0f / L;
    const uint16_t* wrow = a.w + (yok ? y : 0) * a.ldw;
    for (int d4 = tid; d4 < H4; d4 += blockDim.x) {
        f32x4_t e;
        if (MODE == kLLBwd) {
            e = reinterpret_cast<const f32x4_t*>(a.ebuf + int64_t(row) * a.H)[d4];
        } else {
            e = f32x4_t{};
            for (int s = 0; s < a.nsplit; ++s)
                e += s_sc[s] * reinterpret_cast<const f32x4_t*>(a.opart + (int64_t(s) * a.N + m) * a.H)[d4];
            e *= invL;
        }
        if (MODE == kLLFwd) {
            reinterpret_cast<f32x4_t*>(a.ebuf + int64_t(row) * a.H)[d4] = e;
            continue;
        }
        const uint2 wv = reinterpret_cast<const uint2*>(wrow)[d4];
        f32x4_t d;
        d.x = g * (bf_lo(wv.x) - e.x);
        d.y = g * (bf_hi(wv.x) - e.y);
        d.z = g * (bf_lo(wv.y) - e.z);
        d.w = g * (bf_hi(wv.y) - e.w);
        if (!yok) d = f32x4_t{NAN, NAN, NAN, NAN};
        if (a.dh_dtype == TRLX_BF16)
            reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.dh) + int64_t(row) * a.lddh)[d4] =
                make_uint2(pack_bf2(d.x, d.y), pack_bf2(d.z, d.w));
        else
            reinterpret_cast<f32x4_t*>(static_cast<float*>(a.dh) + int64_t(row) * a.lddh)[d4] = d;
    }
}

// ------------------------------------------------------------------ dW
// Workgroup = 64 vocab rows (2 pairs x 32) x one token split; the W fragments stay in
// registers, 32-token tiles of h (+ their lse / g / label) stream through LDS:
//   S[t][v] = Σ_d h[t][d]·W[v][d]        (pair-summed over hidden halves, as in the forward)
//   dS = g_t·(1[y_t = v] − 2^(S·log2e − lse_t·log2e))  -> bf16, the A operand of
//   dW[v][d] += Σ_t dS[t][v]·h[t][d]     (12 d-blocks x 2 k-steps, h read transposed)
template <int KH>
__global__ __launch_bounds__(kLLThreads, 1) void k_lmloss_dw(LmLossArgs a) {
    constexpr int HW = 16 * KH, H = 2 * HW, OB = HW / 32, NI = H / 64;
    constexpr int kStage = kLLRows * H * 2 + 512;  // h tile + {-lse·log2e, g, y, y} x 32 tokens
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage + kLLXchg];
    char* xbuf = smem + 2 * kStage;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, pr = wave >> 1, hh = wave & 1;
    const int hi = lane >> 5, c32 = lane & 31;
    const int nv = a.rows ? *a.nrows : a.N;
    const int nvb = (a.V + kLLVocTile - 1) / kLLVocTile;
    const int vb = int(blockIdx.x) % nvb, ts = int(blockIdx.x) / nvb;
    const int v0 = vb * kLLVocTile + pr * 32;
    const int ntt = (nv + kLLRows - 1) / kLLRows;
    const int t0 = int(int64_t(ts) * ntt / a.tsplit), t1 = int(int64_t(ts + 1) * ntt / a.tsplit);
    bf16x8_t wf[KH];  // B operand of S: lane -> vocab row v0 + c32, hidden hh·HW + 16ks + 8hi + j
    {
        const int vr = v0 + c32;
        if (vr < a.V) {
            const uint16_t* wp = a.w + int64_t(vr) * a.ldw + hh * HW + 8 * hi;
#pragma unroll
            for (int ks = 0; ks < KH; ++ks) wf[ks] = *reinterpret_cast<const bf16x8_t*>(wp + 16 * ks);
        } else {
#pragma unroll
            for (int ks = 0; ks < KH; ++ks) wf[ks] = bf16x8_t{};
        }
    }
    // the two tile rows this lane's DMA pieces fetch (k even: r0, k odd: r0 + 16)
    const int r0 = 4 * wave + (lane >> 4);
    auto tok_row = [&](int m) { const int mc = min(m, nv - 1); return a.rows ? a.rows[mc] : mc; };
    int rowA = 0, rowB = 0;
    if (t0 < t1) {
        rowA = tok_row(t0 * kLLRows + r0);
        rowB = tok_row(t0 * kLLRows + r0 + 16);
    }
    auto issue = [&](int t, char* slot, int ra, int rb) {
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int i = wave + 4 * k;
            ll_piece(slot, i, a.h + int64_t((k & 1) ? rb : ra) * a.ldh, lane);
        }
        if (wave == 0) {  // token scalars: lanes 0-31 -lse·log2e, 32-63 g; then the labels twice
            const int mi = min(t * kLLRows + c32, nv - 1);
            const float* src = hi ? a.gbuf + mi : a.nlse + mi;
            char* sc = slot + kLLRows * H * 2;
            __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)sc, 4, 0, 0);
            __builtin_amdgcn_global_load_lds(a.ybuf + mi, (__attribute__((address_space(3))) void*)(sc + 256), 4, 0, 0);
        }
    };
    f32x16_t D[OB];
#pragma unroll
    for (int b = 0; b < OB; ++b) D[b] = f32x16_t{};
    if (t0 < t1) issue(t0, smem, rowA, rowB);
    for (int t = t0; t < t1; ++t) {
        char* slot = smem + ((t - t0) & 1) * kStage;
        if (t + 1 < t1) {  // next tile's row indices (their loads retire with this tile's pieces)
            rowA = tok_row((t + 1) * kLLRows + r0);
            rowB = tok_row((t + 1) * kLLRows + r0 + 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (t + 1 < t1) issue(t + 1, smem + ((t + 1 - t0) & 1) * kStage, rowA, rowB);
        f32x16_t s = f32x16_t{};
#pragma unroll
        for (int ks = 0; ks < KH; ++ks)
            s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ll_row_frag(slot, lane, hh * HW + 16 * ks), wf[ks], s, 0, 0, 0);
        ll_pair_sum(s, xbuf, wave, lane);
        // s[r] = logit(token t·32 + (r&3) + 8(r>>2) + 4hi, vocab v0 + c32)
        const float* scal = reinterpret_cast<const float*>(slot + kLLRows * H * 2);
        const int* ys = reinterpret_cast<const int*>(slot + kLLRows * H * 2 + 256);
        const int vcol = v0 + c32;
        float ds[16];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int tb = 8 * q + 4 * hi;  // tokens tb .. tb+3 of the tile
            const f32x4_t nl = *reinterpret_cast<const f32x4_t*>(scal + tb);
            const f32x4_t gg = *reinterpret_cast<const f32x4_t*>(scal + 32 + tb);
            const int4 yy = *reinterpret_cast<const int4*>(ys + tb);
            const float nla[4] = {nl.x, nl.y, nl.z, nl.w}, ga[4] = {gg.x, gg.y, gg.z, gg.w};
            const int ya[4] = {yy.x, yy.y, yy.z, yy.w};
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int r = 4 * q + e;
                const bool tok_ok = t * kLLRows + tb + e < nv;
                const float gv = tok_ok ? ga[e] : 0.0f;
                const float pv = exp2_fast(fmaf(s[r], kLog2e, nla[e]));
                ds[r] = gv * ((ya[e] == vcol ? 1.0f : 0.0f) - pv);
            }
        }
        const bf16x8_t db0 = pack8(ds), db1 = pack8(ds + 8);
#pragma unroll
        for (int b = 0; b < OB; ++b) {
            const int dc = hh * HW + 32 * b;
            D[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(db0, ll_tr_frag(slot, lane, 0, dc), D[b], 0, 0, 0);
            D[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(db1, ll_tr_frag(slot, lane, 1, dc), D[b], 0, 0, 0);
        }
    }
    // D[b][r] = dW(vocab v0 + (r&3) + 8(r>>2) + 4hi, hidden hh·HW + 32b + c32)
    const bool part = a.tsplit > 1;  // fp32 partials of this token split, summed by k_lmloss_dw_reduce
#pragma unroll
    for (int r = 0; r < 16; ++r) {
        const int v = v0 + (r & 3) + 8 * (r >> 2) + 4 * hi;
        if (v < a.V) {
            const int64_t o = int64_t(v) * a.lddw + hh * HW + c32;
            if (part || a.dw_dtype == TRLX_F32) {
                float* out = static_cast<float*>(a.dw) + (part ? int64_t(ts) * a.V * a.lddw : 0) + o;
#pragma unroll
                for (int b = 0; b < OB; ++b) out[32 * b] = D[b][r];
            } else {
                uint16_t* out = static_cast<uint16_t*>(a.dw) + o;
#pragma unroll
                for (int b = 0; b < OB; ++b) out[32 * b] = f2bf(D[b][r]);
            }
        }
    }
}

// Fixed-order sum of the token-split dW partials: dw[v][d] = Σ_ts part[ts][v][d].
__global__ __launch_bounds__(256) void k_lmloss_dw_reduce(const float* part, int tsplit, int64_t n, void* dw,
                                                          int dw_dtype, int V, int H, int64_t lddw) {
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t v = i / H, d = i - v * H;
        float acc = 0.0f;
        for (int s = 0; s < tsplit; ++s) acc += part[int64_t(s) * V * H + i];
        st_any(dw, dw_dtype, v * lddw + d, acc);
    }
}

// ------------------------------------------------------------------ mask compaction
// order[0, nv) = rows with mask != 0 in row order, order[nv, N) = ~row of the others, order[N] =
// nv.  Two launches over 1024-row chunks: per-chunk counts, then every chunk sums the counts
// before it (O(N/1024) loads per workgroup) and places its rows.
constexpr int kMaskChunk = 1024;
__global__ __launch_bounds__(256) void k_mask_count(const int64_t* mask, int64_t n, int* cnt) {
    __shared__ int s_red[4];
    const int64_t p0 = int64_t(blockIdx.x) * kMaskChunk;
    int c = 0;
    for (int64_t p = p0 + threadIdx.x; p < min(p0 + kMaskChunk, n); p += blockDim.x) c += mask[p] != 0;
    for (int off = 32; off > 0; off >>= 1) c += __shfl_xor(c, off);
    if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) cnt[blockIdx.x] = s_red[0] + s_red[1] + s_red[2] + s_red[3];
}
__global__ __launch_bounds__(256) void k_mask_place(const int64_t* mask, int64_t n, const int* cnt, int nchunk,
                                                    int* order) {
    __shared__ int s_red[2][4];
    __shared__ int s_scan[256];
    const int tid = threadIdx.x;
    int pre = 0, tot = 0;
    for (int c = tid; c < nchunk; c += blockDim.x) {
        tot += cnt[c];
        pre += c < int(blockIdx.x) ? cnt[c] : 0;
    }
    for (int off = 32; off > 0; off >>= 1) {
        tot += __shfl_xor(tot, off);
        pre += __shfl_xor(pre, off);
    }
    if ((tid & 63) == 0) {
        s_red[0][tid >> 6] = tot;
        s_red[1][tid >> 6] = pre;
    }
    const int64_t p0 = int64_t(blockIdx.x) * kMaskChunk + 4 * tid;  // 4 consecutive rows per thread
    int f[4], loc = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        f[e] = p0 + e < n && mask[p0 + e] != 0;
        loc += f[e];
    }
    s_scan[tid] = loc;
    __syncthreads();
    const int nvalid = s_red[0][0] + s_red[0][1] + s_red[0][2] + s_red[0][3];
    int run = s_red[1][0] + s_red[1][1] + s_red[1][2] + s_red[1][3];
    for (int k = 0; k < tid; ++k) run += s_scan[k];  // valid rows before p0
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        const int64_t p = p0 + e;
        if (p >= n) break;
        if (f[e])
            order[run++] = int(p);
        else
            order[nvalid + int(p - run)] = ~int(p);
    }
    if (blockIdx.x == 0 && tid == 0) order[n] = nvalid;
}

// ------------------------------------------------------------------ host side
static thread_local int g_ll_splits = 0;  // tuning "lmloss_splits" (0 = auto)
static thread_local int g_ll_tsplit = 0;  // tuning "lmloss_dw_tsplit" (0 = auto)

int lmloss_set_tuning(const char* key, int64_t value, bool* handled) {
    const bool sp = key && !__builtin_strcmp(key, "lmloss_splits");
    const bool ts = key && !__builtin_strcmp(key, "lmloss_dw_tsplit");
    *handled = sp || ts;
    if (sp) {
        TRLX_REQUIRE(value >= 0 && value <= kLLMaxSplits, TRLX_ERR_ARG, "lmloss_splits: 0..%d", kLLMaxSplits);
        g_ll_splits = int(value);
    } else if (ts) {
        TRLX_REQUIRE(value >= 0 && value <= 4, TRLX_ERR_ARG, "lmloss_dw_tsplit: 0..4");
        g_ll_tsplit = int(value);
    }
    return TRLX_OK;
}

static size_t ll_align(size_t x) { return (x + 255) & ~size_t(255); }

struct LlWs {
    float* opart;
    float2* mlpart;
    float* xlab;
    float* nlse;
    float* gbuf;
    int* ybuf;
    int* order;
    int* cnt;
    float* dwpart;
};
// Workspace carve-up for N tokens (dwpart only when the dW kernel splits tokens).
static size_t ll_carve(void* base, int64_t N, int64_t H, int64_t V, int tsplit, LlWs* w) {
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* q = p ? p + off : nullptr;
        off += ll_align(bytes);
        return q;
    };
    LlWs t;
    t.opart = reinterpret_cast<float*>(take(size_t(kLLMaxSplits) * N * H * 4));
    t.mlpart = reinterpret_cast<float2*>(take(size_t(kLLMaxSplits) * N * 8));
    t.xlab = reinterpret_cast<float*>(take(size_t(N) * 4));
    t.nlse = reinterpret_cast<float*>(take(size_t(N) * 4));
    t.gbuf = reinterpret_cast<float*>(take(size_t(N) * 4));
    t.ybuf = reinterpret_cast<int*>(take(size_t(N) * 4));
    t.order = reinterpret_cast<int*>(take(size_t(N + 4) * 4));
    t.cnt = reinterpret_cast<int*>(take(size_t((N + kMaskChunk - 1) / kMaskChunk + 1) * 4));
    t.dwpart = reinterpret_cast<float*>(take(tsplit > 1 ? size_t(tsplit) * V * H * 4 : 0));
    if (w) *w = t;
    return off;
}

static int ll_tsplit(int64_t V) {
    if (g_ll_tsplit) return g_ll_tsplit;
    (void)V;
    return 1;
}

static int ll_splits(int64_t N) {
    if (g_ll_splits) return g_ll_splits;
    (void)N;
    return kLLMaxSplits;
}

static int ll_check(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N, int64_t H,
                    int64_t V) {
    TRLX_REQUIRE(hidden && weight, TRLX_ERR_ARG, "NULL hidden / weight");
    TRLX_REQUIRE(N > 0 && V > 0 && N < (int64_t(1) << 31) && V < (int64_t(1) << 31), TRLX_ERR_SHAPE,
                 "bad shape N=%lld V=%lld", (long long)N, (long long)V);
    TRLX_REQUIRE(H == 512 || H == 768, TRLX_ERR_SHAPE,
                 "fused lm_head loss: hidden size %lld not built (512, 768: the h / W halves and the O / dW "
                 "halves of a wave must fit its 512 registers)", (long long)H);
    TRLX_REQUIRE(ldh % 8 == 0 && ldw % 8 == 0 && ldh >= H && ldw >= H, TRLX_ERR_STRIDE,
                 "row strides must be >= H and multiples of 8 elements (16-B rows)");
    TRLX_REQUIRE((reinterpret_cast<uintptr_t>(hidden) & 15) == 0 && (reinterpret_cast<uintptr_t>(weight) & 15) == 0,
                 TRLX_ERR_STRIDE, "hidden / weight must be 16-B aligned");
    return TRLX_OK;
}

template <int KH>
static int ll_launch_fwd(const LmLossArgs& a, hipStream_t s) {
    const int64_t ntt = (a.N + kLLTokTile - 1) / kLLTokTile;
    hipLaunchKernelGGL(k_lmloss_fwd<KH>, dim3(unsigned(ntt * a.nsplit)), dim3(kLLThreads), 0, s, a);
    return check_launch("k_lmloss_fwd");
}
template <int KH>
static int ll_launch_dw(const LmLossArgs& a, hipStream_t s) {
    const int64_t nvb = (a.V + kLLVocTile - 1) / kLLVocTile;
    hipLaunchKernelGGL(k_lmloss_dw<KH>, dim3(unsigned(nvb * a.tsplit)), dim3(kLLThreads), 0, s, a);
    return check_launch("k_lmloss_dw");
}
static int ll_fwd(const LmLossArgs& a, hipStream_t s) {
    return a.H == 512 ? ll_launch_fwd<16>(a, s) : ll_launch_fwd<24>(a, s);
}
static int ll_dw(const LmLossArgs& a, hipStream_t s) {
    return a.H == 512 ? ll_launch_dw<16>(a, s) : ll_launch_dw<24>(a, s);
}

// the common part: shapes, workspace, optional compaction from the mask
static int ll_setup(LmLossArgs& a, const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                    int64_t H, int64_t V, const int64_t* labels, int64_t lb, const int64_t* compact_mask,
                    void* lm_ws, void* dweight, int dw_dtype, int64_t lddw, LlWs& w, hipStream_t s) {
    int rc = ll_check(hidden, ldh, weight, ldw, N, H, V);
    if (rc) return rc;
    TRLX_REQUIRE(labels && lm_ws, TRLX_ERR_ARG, "NULL labels / workspace");
    a.h = static_cast<const uint16_t*>(hidden);
    a.w = static_cast<const uint16_t*>(weight);
    a.ldh = ldh;
    a.ldw = ldw;
    a.N = int(N);
    a.H = int(H);
    a.V = int(V);
    a.labels = labels;
    a.lb = lb;
    a.nsplit = ll_splits(N);
    a.tsplit = ll_tsplit(V);
    ll_carve(lm_ws, N, H, V, a.tsplit, &w);
    a.opart = w.opart;
    a.mlpart = w.mlpart;
    a.xlab = w.xlab;
    a.nlse = w.nlse;
    a.gbuf = w.gbuf;
    a.ybuf = w.ybuf;
    a.dw = a.tsplit > 1 ? static_cast<void*>(w.dwpart) : dweight;
    a.lddw = a.tsplit > 1 ? H : lddw;
    a.dw_dtype = dw_dtype;
    if (compact_mask) {
        const int nchunk = int((N + kMaskChunk - 1) / kMaskChunk);
        hipLaunchKernelGGL(k_mask_count, dim3(nchunk), dim3(256), 0, s, compact_mask, N, w.cnt);
        rc = check_launch("k_mask_count");
        if (rc) return rc;
        hipLaunchKernelGGL(k_mask_place, dim3(nchunk), dim3(256), 0, s, compact_mask, N, w.cnt, nchunk, w.order);
        rc = check_launch("k_mask_place");
        if (rc) return rc;
        a.rows = w.order;
        a.nrows = w.order + N;
    }
    return TRLX_OK;
}

static int ll_dw_finish(const LmLossArgs& a, void* dweight, int dw_dtype, int64_t lddw, const LlWs& w,
                        hipStream_t s) {
    int rc = ll_dw(a, s);
    if (rc || a.tsplit <= 1) return rc;
    const int64_t n = int64_t(a.V) * a.H;
    hipLaunchKernelGGL(k_lmloss_dw_reduce, dim3(2048), dim3(256), 0, s, w.dwpart, a.tsplit, n, dweight, dw_dtype, a.V,
                       a.H, lddw);
    return check_launch("k_lmloss_dw_reduce");
}

}  // namespace trlx

using namespace trlx;

extern "C" int64_t trlx_lmhead_loss_workspace_bytes(int64_t N, int64_t H, int64_t V) {
    return int64_t(ll_carve(nullptr, N, H, V, ll_tsplit(V), nullptr));
}

extern "C" int trlx_ppo_loss_from_hidden(
    const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t B, int64_t T, int64_t H, int64_t V,
    const int64_t* labels, const void* old_lp, int old_dtype, const float* adv_raw, const double* stats, int unbiased,
    const int64_t* mask, const void* values, int v_dtype, const void* old_values, int ov_dtype, const void* returns,
    int r_dtype, float cliprange, float cliprange_value, float vf_coef, float* lp_out, void* dhidden, int64_t lddh,
    int dh_dtype, void* dweight, int dw_dtype, int64_t lddw, float* dvalues, void* workspace, void* lm_workspace,
    void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    LmLossArgs a = {};
    LlWs w;
    const int64_t N = B * T;
    TRLX_REQUIRE(B > 0 && T > 0, TRLX_ERR_SHAPE, "empty rollout batch");
    TRLX_REQUIRE(old_lp && adv_raw && values && old_values && returns && lp_out && dhidden && dweight && dvalues &&
                 workspace, TRLX_ERR_ARG, "NULL argument to trlx_ppo_loss_from_hidden");
    TRLX_REQUIRE(dh_dtype == TRLX_BF16 || dh_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dhidden dtype");
    TRLX_REQUIRE(dw_dtype == TRLX_BF16 || dw_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dweight dtype");
    TRLX_REQUIRE(lddh % 4 == 0 && lddh >= H && lddw >= H, TRLX_ERR_STRIDE, "gradient row strides");
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, 1, mask, lm_workspace, dweight, dw_dtype, lddw, w,
                      s);
    if (rc) return rc;
    Workspace ws;
    carve_ppo_workspace(workspace, B, T, &ws);
    a.mode = kLLPpo;
    a.old_lp = old_lp;
    a.old_dtype = old_dtype;
    a.adv = adv_raw;
    a.stats = stats;
    a.unbiased = unbiased;
    a.mask = mask;
    a.msum = stats ? stats + 3 : nullptr;
    a.msum_host = double(N);
    a.cliprange = cliprange;
    a.lp_out = lp_out;
    a.tokrec = ws.tokrec;
    a.ltok.values = values;
    a.ltok.v_dtype = v_dtype;
    a.ltok.old_values = old_values;
    a.ltok.ov_dtype = ov_dtype;
    a.ltok.returns = returns;
    a.ltok.r_dtype = r_dtype;
    a.ltok.cv = cliprange_value;
    a.ltok.vf_coef = vf_coef;
    a.ltok.dv = dvalues;
    a.dh = dhidden;
    a.lddh = lddh;
    a.dh_dtype = dh_dtype;
    rc = ll_fwd(a, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_lmloss_combine<kLLPpo>, dim3(unsigned(N)), dim3(256), 0, s, a);
    rc = check_launch("k_lmloss_combine");
    if (rc) return rc;
    return ll_dw_finish(a, dweight, dw_dtype, lddw, w, s);
}

extern "C" int trlx_lmhead_logprobs_fwd_saved(const void* hidden, int64_t ldh, const void* weight, int64_t ldw,
                                              int64_t N, int64_t H, int64_t V, const int64_t* labels, int64_t lb,
                                              void* lp_out, int lp_dtype, float* lse_out, float* e_out,
                                              void* lm_workspace, void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    if (N == 0) return TRLX_OK;
    LmLossArgs a = {};
    LlWs w;
    TRLX_REQUIRE(lp_out && lse_out && e_out, TRLX_ERR_ARG, "NULL lp / lse / E output");
    TRLX_REQUIRE(lp_dtype == TRLX_F32 || lp_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "lp dtype");
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, lb, nullptr, lm_workspace, nullptr, TRLX_F32, H,
                      w, s);
    if (rc) return rc;
    a.mode = kLLFwd;
    a.lp = lp_out;
    a.lp_dtype = lp_dtype;
    a.lse_io = lse_out;
    a.ebuf = e_out;
    rc = ll_fwd(a, s);
    if (rc) return rc;
    hipLaunchKernelGGL(k_lmloss_combine<kLLFwd>, dim3(unsigned(N)), dim3(256), 0, s, a);
    return check_launch("k_lmloss_combine");
}

extern "C" int trlx_lmhead_logprobs_bwd(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                        int64_t H, int64_t V, const int64_t* labels, int64_t lb, const void* grad,
                                        int grad_dtype, const float* lse, const float* e, void* dhidden, int64_t lddh,
                                        int dh_dtype, void* dweight, int dw_dtype, int64_t lddw, void* lm_workspace,
                                        void* stream) {
    const hipStream_t s = (hipStream_t)stream;
    if (N == 0) return TRLX_OK;
    LmLossArgs a = {};
    LlWs w;
    TRLX_REQUIRE(grad && lse && e && dhidden && dweight, TRLX_ERR_ARG, "NULL grad / lse / E / gradient output");
    TRLX_REQUIRE(grad_dtype == TRLX_F32 || grad_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "grad dtype");
    TRLX_REQUIRE(dh_dtype == TRLX_BF16 || dh_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dhidden dtype");
    TRLX_REQUIRE(dw_dtype == TRLX_BF16 || dw_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dweight dtype");
    TRLX_REQUIRE(lddh % 4 == 0 && lddh >= H && lddw >= H, TRLX_ERR_STRIDE, "gradient row strides");
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, lb, nullptr, lm_workspace, dweight, dw_dtype, lddw,
                      w, s);
    if (rc) return rc;
    a.mode = kLLBwd;
    a.gin = grad;
    a.gin_dtype = grad_dtype;
    a.lse_io = const_cast<float*>(lse);
    a.ebuf = const_cast<float*>(e);
    a.dh = dhidden;
    a.lddh = lddh;
    a.dh_dtype = dh_dtype;
    hipLaunchKernelGGL(k_lmloss_combine<kLLBwd>, dim3(unsigned(N)), dim3(256), 0, s, a);
    rc = check_launch("k_lmloss_combine");
    if (rc) return rc;
    return ll_dw_finish(a, dweight, dw_dtype, lddw, w, s);
}
