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
#include "row_order.h"

namespace trlx {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef short s16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));

constexpr int kLLRows = 32;            // rows of a staged tile: vocab rows (forward) / tokens (dW)
constexpr int kLLMaxSplits = 8;        // vocab splits of the forward (workspace sizing)
constexpr int kLLTokBlock = 64;        // tokens per forward workgroup (LlGeom: NG = 2 groups of 32)
constexpr float kLLOverflow = 60.0f;
// byte span bound of the hidden / weight buffer resources (below the 0x7ffff000 sentinel)
constexpr int64_t kLLMaxSpan = 0x7fff0000;
// Diagnostic builds only (-DLL_ABLATE=bits, never the shipped library): drop parts of the
// forward's steady-state step to price them — 1 softmax, 2 group-sum exchange, 4 next DMA,
// 8 O product, 16 S product; saved-P stores: 32 no global store, 64 no LDS transpose; the
// saved-P dW kernel: 128 no P loads, 256 no h DMA, 512 dS kept from the first tile.  Results
// are wrong in such a build.
#ifndef LL_ABLATE
#define LL_ABLATE 0
#endif
constexpr int kLLAblate = LL_ABLATE;

// Diagnostic builds only (-DLL_STAMP=1): s_memtime segment sums of the forward's step per wave
// in g_ll_stamps (read by trlx_debug_ll_stamps); no stamp executes in the shipped library.
#ifndef LL_STAMP
#define LL_STAMP 0
#endif
#if LL_STAMP
__device__ unsigned long long g_ll_stamps[1 << 16];
#define LL_TS(v)                                                                              \
    do {                                                                                      \
        __builtin_amdgcn_sched_barrier(0);                                                    \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");             \
        __builtin_amdgcn_sched_barrier(0);                                                    \
    } while (0)
#else
#define LL_TS(v) \
    do {         \
    } while (0)
#endif   // logit - offset bound of the fixed-offset softmax (e^60)

enum LmLossMode { kLLPpo = 0, kLLFwd = 1, kLLBwd = 2 };

struct LmLossArgs {
    const uint16_t* h;   // [N, ldh] bf16 hidden states
    const uint16_t* w;   // [V, ldw] bf16 lm_head weight (nn.Linear layout)
    int64_t ldh, ldw;
    int N, H, V;
    const int64_t* labels;  // [N] (token rows)
    int64_t lb;             // label stride
    // compaction: rows[m] = row of compact token m < *nrows (mask != 0), ~row of the masked
    // ones after them (row_order.h launch_order); NULL = every token, row m
    const int* rows;
    const int* nrows;
    int nsplit;       // vocab splits of the forward: the maximum (nsplit_fixed: exactly)
    int nsplit_fixed;
    float* opart;    // [nsplit][N][H] partial O (compact token index)
    float2* mlpart;  // [nsplit][N] partial (m, l)
    float* trec;     // [N][4] token records {-lse·log2e, d loss / d lp, label bits, 0} (compact;
                     // one 16-B LDS-DMA per lane in the dW kernel)
    int* flags;      // [forward grid][waves] 1 = the wave's fixed offset overflowed (k_lmloss_fwd)
    float* ebuf;     // kLLFwd: E = O / l written here; kLLBwd: read ([N, H], token rows)
    float* lse_io;   // kLLFwd: lse out; kLLBwd: lse in (token rows); may be NULL in kLLPpo
    void* lp;        // lp out (token rows; kLLPpo: fp32 lp_out)
    int lp_dtype;
    const void* gin; // kLLBwd: d loss / d lp (token rows)
    int gin_dtype;
    void* dh;        // [N, lddh] d hidden (token rows)
    int64_t lddh;
    int dh_dtype;
    void* dw;        // [V, lddw] d weight of dw_dtype
    int64_t lddw;
    int dw_dtype;
    // dW grid: dw_full workgroups own a vocab block each over all tokens; the remaining vocab
    // blocks are split tsplit ways over the tokens into fp32 partials ([j][vpw][H]) that
    // k_lmloss_dw_reduce sums in split order (the last, partial round of workgroups)
    int dw_full, tsplit, dw_nblk;
    int dw_vpw;      // vocab rows per dW workgroup (64; the saved-P plan's RW = 2 form: 128)
    float* dwpart;
    // saved-P plan (k_lmloss_dwp): the forward stores its bf16 P tiles in the dW kernel's layout
    // (ll_p_save), the combine a per-(split, token) record {g·e^(m_split − lse), g·(1 − p_y), y, 0}
    uint16_t* pbuf;  // NULL = the recompute plan (k_lmloss_dw)
    int pntt;        // 32-token tiles of the P layout (2·⌈N / 64⌉)
    f32x4_t* prec;   // [kLLMaxSplits][N] (compact token index)
    int ncu;         // compute units (the forward's split choice, ll_fwd_splits)
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
// A [32 rows][H] bf16 tile as H/128 segments of [32 rows][128 columns] (8 KB), each in the
// 8-row x 32-column subtile image of cdna_hip_programming.md T10 (a): 16-B chunk ch of row r sits
// at 2048·(r>>3) + 512·(ch>>2) + 64·(r&7) + 16·((ch&3) ^ ((r>>2)&3)).  The row reads of the
// 32x32x16 operand (32 rows x one 16-B chunk per half-wave) and the transposed reads (4 rows x 16
// columns per 16-lane group) are conflict-free, and the XOR touches only the low 2 bits of the
// chunk: every transposed read of a lane is one of 2 base addresses plus an immediate (column
// block, k-step, segment), every row read one of 2 bases plus an immediate.
__device__ __forceinline__ int ll_off(int r, int d) {
    const int ch = (d >> 3) & 15;
    return (d >> 7) * 8192 + 2048 * (r >> 3) + 512 * (ch >> 2) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3)) +
           ((d & 7) << 1);
}
// The tile row that lane `lane` of DMA piece i fills (piece i: segment i >> 3, 8-row group
// (i & 7) >> 1, subtile pair i & 1).
__device__ __forceinline__ int ll_piece_row(int i, int lane) { return 8 * ((i & 7) >> 1) + ((lane >> 2) & 7); }
// One 1-KB LDS-DMA piece of a tile: lane l lands at the piece's byte 16·l, so it fetches the
// logical chunk that the image puts there.  Buffer-resource form (`row_bytes` = the byte offset
// of the lane's row in the resource): hipcc then tracks these LDS writes like the s2 lm_head
// kernel's and does not put a vmcnt(0) in front of the next LDS read (the flat
// global_load_lds form made every tile wait for the DMA of the NEXT one before its first read).
// The byte offset in the row-major source of the 16 B that lane `lane` of piece i carries.
// The 16x16x32 forms' image (S16) swizzles the 16-B slot with ll16_swz((r>>2)&3) instead of
// (r>>2)&3: their row reads (16 rows x 4 chunks) and transposed reads (rows r, r+4 of a
// subtile in one 32-lane group) were 2-way bank-conflicted on the 32x32 image (PMC:
// SQ_LDS_BANK_CONFLICT = 48 % of the dW kernel's LDS cycles), conflict-free on this one.
__device__ __forceinline__ int ll16_swz(int R) { return (0x78 >> (2 * R)) & 3; }  // 0 2 3 1
__device__ __forceinline__ int ll_piece_src_sw(int i, int row_bytes, int lane, bool s16) {
    const int r = ll_piece_row(i, lane);
    const int sw = s16 ? ll16_swz((r >> 2) & 3) : ((r >> 2) & 3);
    const int ch = 4 * (2 * (i & 1) + (lane >> 5)) + ((lane & 3) ^ sw);
    return row_bytes + (i >> 3) * 256 + ch * 16;
}
__device__ __forceinline__ int ll_piece_src(int i, int row_bytes, int lane) {
    return ll_piece_src_sw(i, row_bytes, lane, false);
}
__device__ __forceinline__ int ll16_piece_src(int i, int row_bytes, int lane) {
    return ll_piece_src_sw(i, row_bytes, lane, true);
}
__device__ __forceinline__ void ll_piece(char* slot, int i, __amdgpu_buffer_rsrc_t rs, int row_bytes, int lane) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(slot + i * 1024), 16,
                                             ll_piece_src(i, row_bytes, lane), 0, 0, 0);
}
__device__ __forceinline__ void ll16_piece(char* slot, int i, __amdgpu_buffer_rsrc_t rs, int row_bytes, int lane) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(slot + i * 1024), 16,
                                             ll16_piece_src(i, row_bytes, lane), 0, 0, 0);
}

// Per-lane byte offsets of the two operand reads inside a staged tile, for a wave whose hidden
// slice starts on a segment boundary (d0 % 128 == 0): every read is then one of these lane bases
// plus a wave-uniform offset d0·64 plus a compile-time immediate (no per-read address VALU).
//   row read, k-step k (32x32x16 A operand by rows: lane -> tile row l&31, columns d0 + 16k + 8hi):
//     d0·64 + (k>>3)·8192 + ((k&7)>>1)·512 + row[k&1]
//   transposed read (k-step s, column block b, tile rows 16s + 4hi + q + 8·p8, columns
//     d0 + 32b + 16(g&1) + 4p for lane 16g + 4q + p):  d0·64 + (b>>2)·8192 + (b&3)·512 + 4096·s + tr[p8]
struct LlLane {
    int row[2];
    int tr[2];
};
__device__ __forceinline__ LlLane ll_lane(int lane) {
    LlLane L;
    const int r = lane & 31, hi = lane >> 5;
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        const int ch = 2 * par + hi;
        L.row[par] = 2048 * (r >> 3) + 64 * (r & 7) + 16 * ((ch & 3) ^ ((r >> 2) & 3));
    }
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int ch = 2 * (g & 1) + (p >> 1);
#pragma unroll
    for (int p8 = 0; p8 < 2; ++p8)
        L.tr[p8] = 2048 * p8 + 64 * (4 * hi + q) + 16 * (ch ^ (hi + 2 * p8)) + 8 * (p & 1);
    return L;
}
__device__ __forceinline__ bf16x8_t ll_row_frag(const char* slice, const LlLane& L, int k) {
    return *reinterpret_cast<const bf16x8_t*>(slice + (k >> 3) * 8192 + ((k & 7) >> 1) * 512 + L.row[k & 1]);
}
__device__ __forceinline__ bf16x8_t ll_tr_frag(const char* slice, const LlLane& L, int s, int b) {
    typedef __attribute__((address_space(3))) s16x4_t lds_s4;
    const char* base = slice + (b >> 2) * 8192 + (b & 3) * 512 + 4096 * s;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + L.tr[0]));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + L.tr[1]));
    const s16x8_t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ bf16x8_t pack8(const float* p) {
    bf16x8_t r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)p[j];
    return r;
}

// Scheduling masks of __builtin_amdgcn_sched_group_barrier (LLVM AMDGPU): VALU, MFMA, any
// VMEM (the LDS-DMA loads), DS read.
constexpr int kSgValu = 0x002, kSgMfma = 0x008, kSgVmem = 0x010, kSgDsRead = 0x100;

// s_waitcnt immediate for vmcnt(n) alone (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt 7,
// lgkmcnt 15): the builtin, unlike inline asm, is seen by the compiler's own wait insertion.
constexpr int ll_vmcnt(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70; }

// max / sum of a value over lanes l and l^32 (one token's two halves), the same bits in both
__device__ __forceinline__ float ll_pair_max(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// max / sum over the four 16-lane rows (lanes l, l^16, l^32, l^48: one token's four lane groups
// in the 16x16x32 forms), the same bits in every lane.  v_permlane16/32_swap are VALU: a
// __shfl_xor is a ds_bpermute, an LDS round trip whose lgkmcnt(0) also drains the operand reads
// in flight.
__device__ __forceinline__ float ll_rows_max(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return ll_pair_max(fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}
__device__ __forceinline__ float ll_pair_sum(float v);
__device__ __forceinline__ float ll_rows_sum(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return ll_pair_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}
__device__ __forceinline__ float ll_pair_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// S tile of one wave over its hidden slice: KS MFMAs whose streamed operand is read by rows.
// Pipelined by sched groups: 3 reads ahead, then (1 MFMA, 1 read, NV vector instructions)
// per gap — left to itself the compiler issued each read right before its MFMA and waited for
// it; NV > 0 pulls independent vector work of the same region (the previous tile's softmax)
// into the MFMA gaps.
template <int KS, int NV>
__device__ __forceinline__ f32x16_t ll_s_product(const char* slice, const LlLane& L, const bf16x8_t* regs) {
    f32x16_t s = f32x16_t{};
    bf16x8_t af[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) af[k] = ll_row_frag(slice, L, k);
#pragma unroll
    for (int k = 0; k < KS; ++k) s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[k], regs[k], s, 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(kSgDsRead, 3, 0);
#pragma unroll
    for (int k = 0; k < KS - 3; ++k) {
        __builtin_amdgcn_sched_group_barrier(kSgMfma, 1, 0);
        __builtin_amdgcn_sched_group_barrier(kSgDsRead, 1, 0);
        if (NV) __builtin_amdgcn_sched_group_barrier(kSgValu, NV, 0);
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        __builtin_amdgcn_sched_group_barrier(kSgMfma, 1, 0);
        if (NV) __builtin_amdgcn_sched_group_barrier(kSgValu, NV, 0);
    }
    return s;
}
// The second product over the wave's slice: OB blocks of 32 hidden columns x 2 k-steps, the
// staged tile read transposed (4 reads per block); LEFT: the register operand is the A operand
// (dW = dSᵀ·h), else the B operand (Oᵀ = Wᵀ·Pᵀ).  Pipelined one block ahead; NDMA > 0 spreads
// that many LDS-DMA pieces of the region (the tile after next) over the MFMA gaps.
template <int OB, bool LEFT, int NDMA>
__device__ __forceinline__ void ll_tr_product(const char* slice, const LlLane& L, bf16x8_t r0, bf16x8_t r1,
                                              f32x16_t* acc) {
    bf16x8_t t[OB][2];
#pragma unroll
    for (int b = 0; b < OB; ++b) {
        t[b][0] = ll_tr_frag(slice, L, 0, b);
        t[b][1] = ll_tr_frag(slice, L, 1, b);
    }
#pragma unroll
    for (int b = 0; b < OB; ++b) {
        if (LEFT) {
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r0, t[b][0], acc[b], 0, 0, 0);
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(r1, t[b][1], acc[b], 0, 0, 0);
        } else {
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t[b][0], r0, acc[b], 0, 0, 0);
            acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(t[b][1], r1, acc[b], 0, 0, 0);
        }
    }
    __builtin_amdgcn_sched_group_barrier(kSgDsRead, 8, 0);
#pragma unroll
    for (int b = 0; b < OB - 2; ++b) {
        __builtin_amdgcn_sched_group_barrier(kSgMfma, 2, 0);
        __builtin_amdgcn_sched_group_barrier(kSgDsRead, 4, 0);
        if (b < NDMA) __builtin_amdgcn_sched_group_barrier(kSgVmem, 1, 0);
    }
    __builtin_amdgcn_sched_group_barrier(kSgMfma, 4, 0);
    constexpr int kRest = NDMA > OB - 2 ? NDMA - (OB - 2) : 0;
    if (kRest) __builtin_amdgcn_sched_group_barrier(kSgVmem, kRest ? kRest : 1, 0);
}

// A workgroup barrier ordering LDS only.  __syncthreads() and an LDS-scope release fence both
// wait for vmcnt(0) — the tile DMAs still in flight are LDS writes too — so the barrier is
// spelled out: this wave's LDS accesses done, then s_barrier (the memory clobber keeps the
// compiler from moving loads / stores across it).
__device__ __forceinline__ void ll_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// The NW waves of a group add their partial S tiles (each over its slice of the hidden
// dimension) through LDS, in the fixed order of their slice index, so every wave of the group
// ends with the same bits.  Write, a workgroup barrier (the caller's), read.
__device__ __forceinline__ void ll_group_write(const f32x16_t& s, char* xbuf, int wave, int lane) {
    f32x4_t* mine = reinterpret_cast<f32x4_t*>(xbuf + wave * 4096);
#pragma unroll
    for (int q = 0; q < 4; ++q) mine[q * 64 + lane] = f32x4_t{s[4 * q], s[4 * q + 1], s[4 * q + 2], s[4 * q + 3]};
}
template <int NW>
__device__ __forceinline__ f32x16_t ll_group_read(const char* xbuf, int wave, int lane) {
    f32x16_t s;
    const f32x4_t* o = reinterpret_cast<const f32x4_t*>(xbuf + (wave - wave % NW) * 4096);
#pragma unroll
    for (int q = 0; q < 4; ++q) {  // own slice read back too: nothing of s stays live across the barrier
        f32x4_t v[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) v[j] = o[j * 256 + q * 64 + lane];  // 4 KB (256 x 16 B) per wave
#pragma unroll
        for (int j = 1; j < NW; ++j) v[0] += v[j];
        s[4 * q] = v[0].x; s[4 * q + 1] = v[0].y; s[4 * q + 2] = v[0].z; s[4 * q + 3] = v[0].w;
    }
    return s;
}
template <int NW>
__device__ __forceinline__ void ll_group_sum(f32x16_t& s, char* xbuf, int wave, int lane) {
    ll_group_write(s, xbuf, wave, lane);
    ll_lds_barrier();
    s = ll_group_read<NW>(xbuf, wave, lane);
}

// Workgroup geometry: NG groups of NW waves; a group owns 32 tokens (forward) / 32 vocab rows
// (dW); wave q of a group holds hidden slice [q·H/NW, (q+1)·H/NW): its h / W fragments
// (H/NW/16 registers x 4) and its slice of O / dW (H/NW/32 blocks x 16 accumulators).
template <int H_, int NG_, int NW_>
struct LlGeom {
    static constexpr int H = H_, NG = NG_, NW = NW_;
    static constexpr int kWaves = NG * NW, kThreads = kWaves * 64;
    static constexpr int HS = H / NW, KS = HS / 16, OB = HS / 32;
    static constexpr int kPieces = H / 16, NI = kPieces / kWaves;  // 1-KB DMA pieces per tile / per wave
    static constexpr int kStage = kLLRows * H * 2;
    static_assert(kPieces % kWaves == 0 && HS % 128 == 0, "geometry: slices start on 128-column segments");
    static_assert(32 * NG == kLLTokBlock, "forward token block (ll_fwd_splits callers)");
    static_assert(kWaves <= 4, "forward overflow flags: 4 words per workgroup (ll_carve)");
};
// 4 waves (one per SIMD, 512 registers each): at H = 768 a wave holds 96 h / W fragment
// registers and 192 accumulators; an 8-wave 4-slice layout (2 waves per SIMD, 256 registers)
// spilled the fragments at every tile, and its 192-column slices do not start on segments.
typedef LlGeom<768, 2, 2> LlG768;
typedef LlGeom<512, 2, 2> LlG512;

// ------------------------------------------------------------------ 16x16x32 operand reads
// Per-lane byte offsets in a staged 32-row tile (subtile image, ll_off) for
// v_mfma_f32_16x16x32_bf16, lane (g, c) = (lane >> 4, lane & 15), q = (lane >> 2) & 3, p = lane & 3:
//   row read of tile row 16mb + c, columns 32ks + 8g (the A operand of an M = rows product):
//     ll16_rb + 4096mb + (ks>>2)·8192 + (ks&3)·512
//   transposed read of rows 4g + q and 16 + 4g + q, columns 16nb + 4p (a K = 32-row operand
//   whose k slots are permuted: slot 8g + j = row 4g + j (j < 4) / 16 + 4g + j − 4 — the
//   rows a lane holds of a 16x16 accumulator pair, see k_lmloss_dw):
//     ll16_trb[nb&1] + (nb>>3)·8192 + ((nb&7)>>1)·512 (+4096)
__device__ __forceinline__ int ll16_rb(int lane) {
    const int g = lane >> 4, c = lane & 15;
    return 2048 * (c >> 3) + 64 * (c & 7) + 16 * (g ^ ll16_swz((c >> 2) & 3));
}
__device__ __forceinline__ int ll16_trb(int lane, int par) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    return 2048 * (g >> 1) + 64 * (4 * (g & 1) + q) + 16 * ((2 * par + (p >> 1)) ^ ll16_swz(g)) + 8 * (p & 1);
}
__device__ __forceinline__ bf16x8_t ll16_row_frag(const char* tile, int rb, int mb, int ks) {
    return *reinterpret_cast<const bf16x8_t*>(tile + rb + 4096 * mb + (ks >> 2) * 8192 + (ks & 3) * 512);
}
__device__ __forceinline__ bf16x8_t ll16_tr_frag(const char* tile, const int* trb, int nb) {
    typedef __attribute__((address_space(3))) s16x4_t lds_s4;
    const char* base = tile + trb[nb & 1] + (nb >> 3) * 8192 + ((nb & 7) >> 1) * 512;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base);
    const s16x4_t hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + 4096));
    const s16x8_t v = {lo.x, lo.y, lo.z, lo.w, hi4.x, hi4.y, hi4.z, hi4.w};
    return __builtin_bit_cast(bf16x8_t, v);
}

// ------------------------------------------------------------------ saved P (the dwp plan)
// The bf16 P tile a 16x16x32 forward wave just formed (lane (g, c): token c of the wave's 16,
// vocab rows 16mb + 4g + r of tile t, element 4mb + r) goes to HBM in the layout the dW kernel
// consumes as its A operand, so k_lmloss_dwp loads one 16-B chunk per lane and never recomputes
// S:  pbuf[vb = t/2][token tile tt][dW wave 2(t&1) + hv][dW lane (g, c)][16 B] holds vocab row
// 16hv + c of the tile for tokens 8g..8g+7 of the 32-token tile (k_lmloss_dwp's k slots: slot j
// of lane group g = token 8g + j).  Lane groups g = 2·half, 2·half + 1 come from the forward
// wave holding the tile's tokens 16·half..16·half+15, so every forward lane stores one whole
// 16-B chunk (512 contiguous bytes per wave and dW wave).  The transpose runs through a
// per-wave 16 x 32 LDS image (token rows of kLLPRow bytes): two ds_read_b64_tr_b16 give lane
// (g, c) column 16·(g >> 1) + c, token rows 8·(g & 1) + 0..3 and + 4..7 (T10).
constexpr int kLLPRow = 72;
__device__ __forceinline__ s16x8_t ll_p_stage(char* pscr, bf16x8_t pb, int lane) {
    typedef __attribute__((address_space(3))) s16x4_t lds_s4;
    const int g = lane >> 4, c = lane & 15, q = (lane >> 2) & 3, p = lane & 3;
    const s16x8_t v = __builtin_bit_cast(s16x8_t, pb);
    *reinterpret_cast<s16x4_t*>(pscr + kLLPRow * c + 8 * g) = s16x4_t{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<s16x4_t*>(pscr + kLLPRow * c + 32 + 8 * g) = s16x4_t{v[4], v[5], v[6], v[7]};
    const char* rd = pscr + kLLPRow * (8 * (g & 1) + q) + 32 * (g >> 1) + 8 * p;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)rd);
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(rd + 4 * kLLPRow));
    return s16x8_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
}
// The same transpose read straight from the wave's O-exchange slot (the 16 B of P a lane wrote
// at slot + 16·lane, LL_FWD_OXCH): the 8-B chunk (token R, lane group g', block mb) that the image
// above holds at kLLPRow·R + 8g' + 32mb sits at 16·(16g' + R) + 8mb, so the two tr reads take
// those addresses and no image is written (4-way bank conflicts on 2 reads a tile instead).
__device__ __forceinline__ s16x8_t ll_p_stage_slot(const char* slot, int lane) {
    typedef __attribute__((address_space(3))) s16x4_t lds_s4;
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const char* rd = slot + 16 * (16 * p + 8 * (g & 1) + q) + 8 * (g >> 1);
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)rd);
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(rd + 64));
    return s16x8_t{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
}
__device__ __forceinline__ void ll_p_store(const LmLossArgs& a, const s16x8_t& v, int t, int tt, int half,
                                           int lane) {
    const int g = lane >> 4, c = lane & 15;
    char* dst = reinterpret_cast<char*>(a.pbuf) +
                ((int64_t(t >> 1) * a.pntt + tt) * 4 + 2 * (t & 1) + (g >> 1)) * 1024 +
                16 * (16 * (2 * half + (g & 1)) + c);
    *reinterpret_cast<s16x8_t*>(dst) = v;
}

// Vocab splits of the forward for ntb live token blocks: the count (<= a.nsplit) whose last
// round of workgroups is fullest — cost = ceil(ntb·ns / ncu) / ns rounds of one whole-vocab
// block; ties go to more splits.  A pure function of the device-side token count, so the
// combine recomputes it.
__device__ __forceinline__ int ll_fwd_splits(const LmLossArgs& a, int ntb) {
    if (a.nsplit_fixed) return a.nsplit;
    int best = 1;
    float bc = 3.0e38f;
    for (int ns = 1; ns <= a.nsplit; ++ns) {
        const float c = float((ntb * ns + a.ncu - 1) / a.ncu) / float(ns);
        if (c <= bc) {
            bc = c;
            best = ns;
        }
    }
    return best;
}

// ------------------------------------------------------------------ forward (flash-O)
// Workgroup = NG·32 tokens x one vocab split; wave (group g, slice q).  Per 32-row vocab tile:
//   S^T[v][t] = Σ_d W[v][d]·h[t][d]   (KS MFMAs over the wave's hidden slice, group sum in LDS)
//   P = exp(S - offset) per token (lanes t and t^32 hold its 32 values), Σ P
//   O^T[d][t] += Σ_v W[v][d]·P[t][v] (OB d-blocks x 2 k-steps: W read transposed, P = the S
//   accumulator converted to bf16 as the B operand): each lane's O registers are ONE token's.
// One wave per SIMD, so the softmax's vector work only overlaps matrix work of the SAME wave:
// the loop is software-pipelined one tile deep — step t runs S(t+1)'s MFMAs with softmax(t)'s
// vector instructions in their gaps (sched groups), then O(t)'s MFMAs with tile t+2's DMA in
// theirs.  Three 48-KB stages (t, t+1 read; t+2 landing) + the 16-KB group-sum exchange = the
// whole 160 KB.  The label logit is not picked here: k_lmloss_combine dots h with W[y].
template <class G, bool RESTART>
__device__ __forceinline__ void ll_fwd_block(const LmLossArgs& a, char* smem, int lin, int ntb, int nsplit, int nv) {
    constexpr int HS = G::HS, KS = G::KS, OB = G::OB, NI = G::NI, kStage = G::kStage;
    char* xbuf = smem + 3 * kStage;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), grp = wave / G::NW, sq = wave % G::NW;
    const int hi = lane >> 5, c32 = lane & 31;
    const LlLane LL = ll_lane(lane);
    const int split = lin / ntb, mt = lin - split * ntb;
    const int m0 = mt * 32 * G::NG;
    const int tm = m0 + grp * 32 + c32;
    const bool valid = tm < nv;
    const int tc = valid ? tm : nv - 1;
    const int row = a.rows ? a.rows[tc] : tc;
    bf16x8_t hf[KS];  // B operand of S^T: lane -> token c32, hidden sq·HS + 16ks + 8hi + j
    {
        const uint16_t* hp = a.h + int64_t(row) * a.ldh + sq * HS + 8 * hi;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) hf[ks] = *reinterpret_cast<const bf16x8_t*>(hp + 16 * ks);
    }
    const int nvt = (a.V + kLLRows - 1) / kLLRows;
    const int t0 = int(int64_t(split) * nvt / nsplit), t1 = int(int64_t(split + 1) * nvt / nsplit);
    // W rows by buffer loads: rows past V read zeros (range check), their logits are masked.
    // A tile index past the split gives an out-of-range offset: the pieces fetch nothing.
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, uint32_t(int64_t(a.V) * a.ldw * 2));
    auto issue = [&](int t, char* slot) __attribute__((always_inline)) {
        const bool live = t < t1;
#pragma unroll
        for (int k = 0; k < NI; ++k) {
            const int i = wave + G::kWaves * k;
            const int off = (t * kLLRows + ll_piece_row(i, lane)) * int(a.ldw) * 2;
            ll_piece(slot, i, rw, live ? off : int(0x7ffff000), lane);
        }
    };
    // The exponent offset of a token is FIXED for the whole split: the first tile's max (no
    // online rescale of O — a rescale of the accumulators in a branch made the compiler spill
    // them, and a max that moves by < kLLOverflow leaves every term < e^60, in fp32 and bf16
    // range).  If some token's logits exceed its offset by more than that, the wave flags
    // itself and records the true maxima; the RESTART launch reruns the flagged workgroups with
    // offset = the true max (never on realistic logits; the others exit at once).  A second
    // launch rather than a loop around this one: with the loop, hipcc no longer told the next
    // tile's DMA apart from this tile's reads and waited for the DMA before every tile.
    float mfix = -INFINITY, mtrue = -INFINITY, lrun = 0.0f;
    if (RESTART) mfix = a.mlpart[int64_t(split) * a.N + tc].x;  // the true max pass 0 found
    f32x16_t O[OB];
#pragma unroll
    for (int b = 0; b < OB; ++b) O[b] = f32x16_t{};
    bool bad = false;
    // softmax of tile t's summed S (s[r] = logit(token c32, vocab t·32 + (r&3) + 8(r>>2) + 4hi)):
    // branch-free so it shares a scheduling region with the next tile's MFMAs
    // (only the vocab's last tile can be partial: it is the last split's last tile, whose
    // softmax runs after the loop — MASK there only)
    auto softmax = [&](f32x16_t s, int t, bf16x8_t& pb0, bf16x8_t& pb1, auto mask_tag) __attribute__((always_inline)) {
        constexpr bool MASK = decltype(mask_tag)::value;
        float mx = -INFINITY;
        if (MASK) {
            const int lim = a.V - t * kLLRows - 4 * hi;  // rows with (r&3) + 8(r>>2) < lim exist
#pragma unroll
            for (int r = 0; r < 16; ++r) s[r] = (r & 3) + 8 * (r >> 2) < lim ? s[r] : -INFINITY;
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, s[r]);
        mx = ll_pair_max(mx);
        if (!RESTART) {
            mtrue = fmaxf(mtrue, mx);
            mfix = t == t0 ? mx : mfix;
            bad = bad || mx > mfix + kLLOverflow;
        }
        const float nm = -mfix * kLog2e;
        float p[16];
        float ls = 0.0f;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            p[r] = exp2_fast(fmaf(s[r], kLog2e, nm));
            ls += p[r];
        }
        lrun += ls;
        pb0 = pack8(p);
        pb1 = pack8(p + 8);
    };
    // step t (t + 1 < t1): the four LDS regions as __restrict__ parameters of an inlined call,
    // so the compiler's alias scopes tell tile t+2's DMA (fut) apart from this step's reads
    // One DMA piece k (of NI) of tile t into slot (an out-of-range offset past the split).
    auto issue_piece = [&](int t, char* slot, int k) __attribute__((always_inline)) {
        const int i = wave + G::kWaves * k;
        const int off = (t * kLLRows + ll_piece_row(i, lane)) * int(a.ldw) * 2;
        ll_piece(slot, i, rw, t < t1 ? off : int(0x7ffff000), lane);
    };
    // The step's schedule is written out gap by gap, each gap fenced (sched_barrier): the
    // compiler's own interleave left the softmax's vector work and the DMA issue in segments of
    // their own (stamps: 1529 cycles for S + softmax, 678 for the exchange write + 12 DMA issues,
    // against 768 of MFMA each side).
    //   S phase, gap k (KS gaps): row read k+4 | MFMA k of S(t+1) | softmax(t) chunk k
    //   O phase, gap i (2·OB gaps, k-step-major): tr read i+4 | MFMA i of O(t) | P's second half
    //     packed (i = 0), S(t+1)'s partial written (i = 2..5), at i = OB the exchange barrier and
    //     the partner's partial read (summed after the loop, consumed by the next step)
    //   and every 3rd gap from the step's start one LDS-DMA piece of tile t+2 (the last ones early
    //   in the O phase, so they land before the next step's wait): a piece is 1 KB through the
    //   CU's vector-memory path, and bunched pieces stall their wave's issue (stamps: 12 in a row
    //   cost ~600 cycles)
    f32x16_t s;  // summed S of the tile whose softmax comes next
#if LL_STAMP
    unsigned long long stamp[8] = {};
#endif
    auto step = [&](const char* __restrict__ cur, const char* __restrict__ nx, char* __restrict__ fut,
                    char* __restrict__ xb, int t) __attribute__((always_inline)) {
        unsigned long long ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0, ts4 = 0, ts5 = 0, ts6 = 0;
        LL_TS(ts0);
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(0));  // this wave's pieces of tile t+1
        ll_lds_barrier();  // every wave's; every wave is done with xb and with tile t-1
        LL_TS(ts1);
        // ---- S phase
        const char* ns = nx + sq * HS * 64;
        constexpr int PF = 4;
        bf16x8_t af[KS];
#pragma unroll
        for (int k = 0; k < PF; ++k) af[k] = ll_row_frag(ns, LL, k);
        f32x16_t s1 = f32x16_t{};
        float m0, m1, m2, m3, m4, m5, mx = 0.0f, nm = 0.0f, ls = 0.0f;
        float p[16];
#pragma unroll
        for (int k = 0; k < KS; ++k) {
            if (k + PF < KS) af[k + PF] = ll_row_frag(ns, LL, k + PF);
            s1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[k], hf[k], s1, 0, 0, 0);
            if (k == 0) {
                m0 = fmaxf(fmaxf(s[0], s[1]), s[2]);
                m1 = fmaxf(fmaxf(s[3], s[4]), s[5]);
            } else if (k == 1) {
                m2 = fmaxf(fmaxf(s[6], s[7]), s[8]);
                m3 = fmaxf(fmaxf(s[9], s[10]), s[11]);
            } else if (k == 2) {
                m4 = fmaxf(fmaxf(s[12], s[13]), s[14]);
                m5 = fmaxf(fmaxf(m0, m1), s[15]);
            } else if (k == 3) {
                mx = fmaxf(fmaxf(fmaxf(m2, m3), m4), m5);
            } else if (k == 4) {
                mx = ll_pair_max(mx);
                if (!RESTART) {
                    mtrue = fmaxf(mtrue, mx);
                    mfix = t == t0 ? mx : mfix;
                    bad = bad || mx > mfix + kLLOverflow;
                }
                nm = -mfix * kLog2e;
            } else {
                const int rlo = (k - 5) * 16 / (KS - 5), rhi = (k - 4) * 16 / (KS - 5);
#pragma unroll
                for (int r = rlo; r < rhi; ++r) {
                    p[r] = exp2_fast(fmaf(s[r], kLog2e, nm));
                    ls += p[r];
                }
            }
            if (k % 3 == 1 && k / 3 < NI && !(kLLAblate & 4)) issue_piece(t + 2, fut, k / 3);
            __builtin_amdgcn_sched_barrier(0);
        }
        lrun += ls;
        const bf16x8_t pb0 = pack8(p);
        bf16x8_t pb1;
        LL_TS(ts2);
        LL_TS(ts3);
        // ---- O phase
        const char* cs = cur + sq * HS * 64;
        constexpr int PFO = 4;
        bf16x8_t tf[2 * OB];
#pragma unroll
        for (int i = 0; i < PFO; ++i) tf[i] = ll_tr_frag(cs, LL, i / OB, i % OB);
        f32x4_t xv[4][G::NW];
#pragma unroll
        for (int i = 0; i < 2 * OB; ++i) {
            if (i + PFO < 2 * OB) tf[i + PFO] = ll_tr_frag(cs, LL, (i + PFO) / OB, (i + PFO) % OB);
            if (i == 0) pb1 = pack8(p + 8);
            const int b = i % OB;
            O[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf[i], i < OB ? pb0 : pb1, O[b], 0, 0, 0);
            if (i >= 2 && i < 6) {  // S(t+1)'s partial: quarter i-2
                const int q = i - 2;
                reinterpret_cast<f32x4_t*>(xb + wave * 4096)[q * 64 + lane] =
                    f32x4_t{s1[4 * q], s1[4 * q + 1], s1[4 * q + 2], s1[4 * q + 3]};
            }
            if ((KS + i) % 3 == 1 && (KS + i) / 3 < NI && !(kLLAblate & 4)) issue_piece(t + 2, fut, (KS + i) / 3);
            if (i == OB) {
                LL_TS(ts4);
                ll_lds_barrier();  // every wave's partial written
                LL_TS(ts5);
                const f32x4_t* o = reinterpret_cast<const f32x4_t*>(xb + (wave - wave % G::NW) * 4096);
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int j = 0; j < G::NW; ++j) xv[q][j] = o[j * 256 + q * 64 + lane];
            }
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            f32x4_t v = xv[q][0];
#pragma unroll
            for (int j = 1; j < G::NW; ++j) v += xv[q][j];
            s[4 * q] = v.x; s[4 * q + 1] = v.y; s[4 * q + 2] = v.z; s[4 * q + 3] = v.w;
        }
        LL_TS(ts6);
#if LL_STAMP
        stamp[0] += ts1 - ts0;
        stamp[1] += ts2 - ts1;
        stamp[2] += ts3 - ts2;
        stamp[3] += ts4 - ts3;
        stamp[4] += ts5 - ts4;
        stamp[5] += ts6 - ts5;
        stamp[6] += 1;
#endif
        (void)ts0, (void)ts1, (void)ts2, (void)ts3, (void)ts4, (void)ts5, (void)ts6;
    };
    if (t0 < t1) {
        char* c0 = smem;
        char* c1 = smem + kStage;
        char* c2 = smem + 2 * kStage;
        issue(t0, c0);
        issue(t0 + 1, c1);
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(NI));  // tile t0 (t0+1 may fly)
        ll_lds_barrier();
        s = ll_s_product<KS, 0>(c0 + sq * HS * 64, LL, hf);
        ll_group_write(s, xbuf, wave, lane);
        ll_lds_barrier();
        s = ll_group_read<G::NW>(xbuf, wave, lane);
        for (int t = t0; t + 1 < t1; ++t) {
            step(c0, c1, c2, xbuf, t);
            char* c = c0;
            c0 = c1;
            c1 = c2;
            c2 = c;
        }
        bf16x8_t pb0, pb1;  // the last tile: its softmax and O product
        softmax(s, t1 - 1, pb0, pb1, std::true_type{});
        ll_tr_product<OB, false, 0>(c0 + sq * HS * 64, LL, pb0, pb1, O);
    }
    // the first launch flags an overflowed wave and records the true maxima as its m (its O / l
    // are then discarded: the restart launch reruns the workgroup).  A flag word per wave: a
    // workgroup-wide vote (__syncthreads_or) here brought back a per-tile DMA wait.
#if LL_STAMP
    if (lane == 0 && !RESTART && lin * G::kWaves + wave < (1 << 13))
        for (int k = 0; k < 8; ++k) g_ll_stamps[(lin * G::kWaves + wave) * 8 + k] = stamp[k];
#endif
    bool any = false;
    if (!RESTART) {
        any = __any(bad);
        if (lane == 0) a.flags[lin * G::kWaves + wave] = any;
    }
    const float mrun = any ? mtrue : mfix;
    const float ltok = ll_pair_sum(lrun);
    if (valid) {
        // O[b][r] = O(token c32, hidden sq·HS + 32b + (r&3) + 8(r>>2) + 4hi)
        float* op = a.opart + (int64_t(split) * a.N + tm) * a.H + sq * HS + 4 * hi;
#pragma unroll
        for (int b = 0; b < OB; ++b)
#pragma unroll
            for (int q = 0; q < 4; ++q)
                *reinterpret_cast<f32x4_t*>(op + 32 * b + 8 * q) =
                    f32x4_t{O[b][4 * q], O[b][4 * q + 1], O[b][4 * q + 2], O[b][4 * q + 3]};
        if (sq == 0 && hi == 0) a.mlpart[int64_t(split) * a.N + tm] = make_float2(mrun, ltok);
    }
}

// ------------------------------------------------------------------ forward, 16x16x32 form
// A workgroup = 64 tokens (four blocks of 16, one softmax per wave: block w) x one vocab split;
// h fragments 96 registers, O 192 at H = 768.  Without the two splits below (LL_FWD_SPAIR,
// LL_FWD_OXCH — both on by default) a wave computes S and O of its own block over the whole H,
// the k_lmloss_dw layout with the roles swapped.  Per 32-row W tile, on v_mfma_f32_16x16x32_bf16:
//   S[v][t] = Σ_d W[v][d]·h[t][d]     2 vocab blocks x H/32 k-steps (W rows the A operand, the
//                                     h fragments the B operand): lane (g, c) ends with vocab
//                                     rows 16mb + 4g + r of token c
//   P = 2^(S·log2e − offset·log2e)    8 values a lane; the token's offset is the first tile's
//                                     max over its 4 lanes (g), fixed for the split, as ll_fwd_block
//   Oᵀ[d][t] += Σ_v W[v][d]·P[v][t]   H/16 column blocks x one permuted k-step (W read
//                                     transposed: the A operand; the lane's own 8 P values: B)
// Software-pipelined one tile deep over a 3-stage ring: S(t+1) beside softmax(t) and tile t+2's
// DMA, one barrier, O(t) (DESIGN.md §3 "The forward at HEAD").
#ifndef LL_FWD_PIECE_GAP
#define LL_FWD_PIECE_GAP 2
#endif
#ifndef LL_FWD_PIECE_OFF
#define LL_FWD_PIECE_OFF 1
#endif
#ifndef LL_FWD_PSTAGE_GAP
#define LL_FWD_PSTAGE_GAP 30
#endif
// O exchange (default): the O product splits the hidden columns over the four waves instead of
// the tokens — wave w accumulates d blocks 16i + 4w + j (i < H/256, j < 4) for all 64 tokens of
// the workgroup, each transposed W fragment feeding four MFMAs (one per token block) — so a wave
// reads a quarter of the tile transposed (12 instead of 48 KB at H = 768) plus the four waves'
// P (1 KB each, written to LDS after the softmax, read after a mid-step barrier)
#ifndef LL_FWD_OXCH
#define LL_FWD_OXCH 1
#endif
// W row fragments in flight in the S loop
#ifndef LL_FWD_PF
#define LL_FWD_PF 4
#endif
// S split over the hidden halves of a wave pair (needs the O exchange): wave w = (hidden half
// w & 1, token pair w >> 1) accumulates partial S over its half for BOTH token blocks of the
// pair (h fragments: 2 blocks x H/2 = the same 96 registers), so each W row fragment feeds two
// MFMAs and a wave reads half the tile by rows; the partner's partial of the wave's own block
// comes through LDS (written in the O loop, read after the next step's barrier)
#ifndef LL_FWD_SPAIR
#define LL_FWD_SPAIR 1
#endif
// How tile t+2 reaches LDS in step t: 0 = LDS-DMA pieces in the S loop's gaps; 1 = LDS-DMA
// pieces in the O exchange loop's gaps; 2 = register-staged (buffer loads in the S loop's gaps,
// ds_write_b128 in the O exchange loop's) — 1 and 2 measured slower (profiles/r05f_fwd_oxch.txt)
#ifndef LL_FWD_FILL
#define LL_FWD_FILL 0
#endif
// SAVEP with the O exchange: the saved-P transpose read from the exchange slot (ll_p_stage_slot)
#ifndef LL_FWD_PSLOT
#define LL_FWD_PSLOT 1
#endif
template <class G, bool RESTART, bool SAVEP>
__device__ __forceinline__ void ll_fwd16_block(const LmLossArgs& a, char* smem, int lin, int ntb, int nsplit,
                                               int nv) {
    constexpr int H = G::H, KS = H / 32, DB = H / 16, NI = G::NI, kStage = G::kStage;
    constexpr int NG = 2 * KS;  // S-phase gaps
    // tile t+2's DMA pieces: every kPG-th gap of the step's S + O sequence from gap kPO
    constexpr int kPG = LL_FWD_PIECE_GAP, kPO = LL_FWD_PIECE_OFF;
    static_assert(kPO >= 0, "the DMA piece offset (the first piece's gap)");
    // piece i of tile t+2 in gap kPO + kPG·i
    auto piece_at = [](int k) { return k >= kPO && (k - kPO) % kPG == 0 && (k - kPO) / kPG < NI; };
    // SAVEP: the gap (of the S + O sequence) that stages P through LDS (after the pack at 11;
    // with LL_FWD_SPAIR the O loop's first gap instead)
    constexpr int kPS = LL_FWD_PSTAGE_GAP;
    static_assert(kPS > 11 && kPS < NG + DB, "the P staging gap");
    static_assert(NG >= 20, "the P-save gaps");
    constexpr bool OX = LL_FWD_OXCH;
    constexpr int OI = DB / 16, OF = 4 * OI;  // OX: the wave's 4-block d groups / its W^T fragments
    static_assert(!OX || (DB % 16 == 0 && G::kWaves == 4 && kLLTokBlock == 64), "O exchange geometry");
    static_assert(!OX || (kPG * (NI - 1) + kPO < NG && kPS < NG), "O exchange: the pieces and the P staging in the S loop");
    constexpr int kFill = LL_FWD_FILL;
    static_assert(kFill == 0 || (OX && OF == NI), "fills in the O exchange loop: one piece per gap");
    constexpr bool SP = LL_FWD_SPAIR;
    constexpr int KH = KS / 2;  // SP: k-steps of a hidden half
    static_assert(!SP || (OX && KH % 4 == 0 && kFill == 0), "S pair split: the O exchange, whole 128-column segments");
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // SAVEP: this wave's P transpose image (the exchange region, unused by this form) and its
    // place in the dW layout (ll_p_stage / ll_p_store)
    char* pscr = smem + 3 * kStage + wave * 4096;
    // OX: this wave's P for the exchange (past the transpose image) and the lane's read of token
    // block tb's (+ 4096·tb)
    char* xch = pscr + 2048 + 16 * (lane & 63);
    const char* xrd = smem + 3 * kStage + 2048 + 16 * (lane & 63);
    constexpr bool PSL = OX && LL_FWD_PSLOT;  // the saved-P transpose from the exchange slot
    static_assert(!PSL || kPS > 12, "the saved-P transpose after the exchange slot's write (gap 12)");
    auto p_stage = [&](const bf16x8_t& pbv) __attribute__((always_inline)) {
        if constexpr (PSL)
            return ll_p_stage_slot(pscr + 2048, lane);
        else
            return ll_p_stage(pscr, pbv, lane);
    };
    const int g = lane >> 4, c = lane & 15;
    const int split = lin / ntb, mt = lin - split * ntb;
    const int tm = mt * kLLTokBlock + wave * 16 + c;  // this lane's token (compact index)
    const int ptt = 2 * mt + (wave >> 1), phalf = wave & 1;
    const bool valid = tm < nv;
    const int tc = valid ? tm : nv - 1;
    const int row = a.rows ? a.rows[tc] : tc;
    // B operand of S: lane (g, c) -> h[token c][32ks + 8g .. +7]; SP: hf[ks] own token block,
    // hf[KH + ks] the partner's (wave ^ 1), columns (H/2)(wave & 1) + 32ks + 8g
    bf16x8_t hf[KS];
    if constexpr (SP) {
        const int tmp = mt * kLLTokBlock + (wave ^ 1) * 16 + c;
        const int tcp = tmp < nv ? tmp : nv - 1;
        const int rowp = a.rows ? a.rows[tcp] : tcp;
        const uint16_t* hp = a.h + int64_t(row) * a.ldh + (H / 2) * (wave & 1) + 8 * g;
        const uint16_t* hq = a.h + int64_t(rowp) * a.ldh + (H / 2) * (wave & 1) + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KH; ++ks) {
            hf[ks] = *reinterpret_cast<const bf16x8_t*>(hp + 32 * ks);
            hf[KH + ks] = *reinterpret_cast<const bf16x8_t*>(hq + 32 * ks);
        }
    } else {
        const uint16_t* hp = a.h + int64_t(row) * a.ldh + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) hf[ks] = *reinterpret_cast<const bf16x8_t*>(hp + 32 * ks);
    }
    // SP: this wave's half of the W rows (rb + the half's segments) and the partner's partial S
    const int rbh = ll16_rb(lane) + KS * 1024 * (wave & 1);
    const char* sxr = smem + 3 * kStage + (wave ^ 1) * 4096 + 16 * (lane & 63);
    char* sxw = pscr + 16 * (lane & 63);
    const int nvt = (a.V + kLLRows - 1) / kLLRows;
    const int t0 = int(int64_t(split) * nvt / nsplit), t1 = int(int64_t(split + 1) * nvt / nsplit);
    const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w, uint32_t(int64_t(a.V) * a.ldw * 2));
    auto issue_piece = [&](int t, char* slot, int k) __attribute__((always_inline)) {
        const int i = wave + G::kWaves * k;
        const int off = (t * kLLRows + ll_piece_row(i, lane)) * int(a.ldw) * 2;
        ll16_piece(slot, i, rw, t < t1 ? off : int(0x7ffff000), lane);
    };
    auto load_piece = [&](int t, int k) __attribute__((always_inline)) {
        const int i = wave + G::kWaves * k;
        const int off = (t * kLLRows + ll_piece_row(i, lane)) * int(a.ldw) * 2;
        return __builtin_amdgcn_raw_buffer_load_b128(rw, ll16_piece_src(i, t < t1 ? off : int(0x7ffff000), lane), 0, 0);
    };
    const int rb = ll16_rb(lane);
    const int trb[2] = {ll16_trb(lane, 0), ll16_trb(lane, 1)};
    // OX: W^T fragment (i, j) = d block 16i + 4·wave + j: ll16_tr_frag's offset with the wave's
    // part folded into the lane bases (a multiple of 256 B: the conflict-free banking unchanged)
    const int trx[2] = {trb[0] + 8192 * (wave >> 1) + 1024 * (wave & 1), trb[1] + 8192 * (wave >> 1) + 1024 * (wave & 1)};
    auto ox_frag = [&](const char* tile, int f) __attribute__((always_inline)) {
        typedef __attribute__((address_space(3))) s16x4_t lds_s4;
        const int i = f >> 2, j = f & 3;
        const char* base = tile + trx[j & 1] + 16384 * i + 512 * (j >> 1);
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)base);
        const s16x4_t hi4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + 4096));
        const s16x8_t v = {lo.x, lo.y, lo.z, lo.w, hi4.x, hi4.y, hi4.z, hi4.w};
        return __builtin_bit_cast(bf16x8_t, v);
    };
    float mfix = -INFINITY, mtrue = -INFINITY, lrun = 0.0f;
    if (RESTART) mfix = a.mlpart[int64_t(split) * a.N + tc].x;  // the true max pass 0 found
    bool bad = false;
    f32x4_t O[DB];  // Oᵀ[16nb + 4g + r][token c]; OX: O[4f + tb] = Oᵀ[d block of fragment f][token block tb]
#pragma unroll
    for (int nb = 0; nb < DB; ++nb) O[nb] = f32x4_t{};
    // OX: O(t) over the wave's d groups for the four token blocks, after the exchange barrier
    // (the first PFX fragments come in tf: read before the exchange barrier, they depend on the
    // tile only)
    constexpr int PFX = 2;
    auto ox_product = [&](const char* tile, bf16x8_t (&tf)[OF], int gbase, auto&& gap) __attribute__((always_inline)) {
        bf16x8_t px[4];
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) px[tb] = *reinterpret_cast<const bf16x8_t*>(xrd + 4096 * tb);
#pragma unroll
        for (int f = 0; f < OF; ++f) {
            if (f + PFX < OF) tf[f + PFX] = ox_frag(tile, f + PFX);
#pragma unroll
            for (int tb = 0; tb < 4; ++tb)
                O[4 * f + tb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tf[f], px[tb], O[4 * f + tb], 0, 0, 0);
            gap(gbase + f);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    f32x4_t s[2];  // S of the tile whose softmax comes next (SP: the wave's partial of its own block)
    f32x4_t so[2];  // SP: the partial of the partner's block (to the exchange)
    float x[8], pr[8], m4 = 0.0f, nm = 0.0f, ls = 0.0f;
    // softmax of tile t in chunks (chunk k of 12): 0 = the lane's max + the token max over its
    // four lanes, 1 = offset / overflow flag, 2..9 = one exp each, 10 = the row sum
    auto sm_chunk = [&](int k, int t, auto mask_tag) __attribute__((always_inline)) {
        constexpr bool MASK = decltype(mask_tag)::value;
        if (k == 0) {
            const int lim = a.V - t * kLLRows - 4 * g;  // vocab row 16mb + 4g + r exists iff 16mb + r < lim
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const float v = s[e >> 2][e & 3];
                x[e] = (!MASK || 16 * (e >> 2) + (e & 3) < lim) ? v : -INFINITY;
            }
            const float lm = fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])),
                                   fmaxf(fmaxf(x[4], x[5]), fmaxf(x[6], x[7])));
            m4 = ll_rows_max(lm);
        } else if (k == 1) {
            if (!RESTART) {
                mtrue = fmaxf(mtrue, m4);
                mfix = t == t0 ? m4 : mfix;
                bad = bad || m4 > mfix + kLLOverflow;
            }
            nm = -mfix * kLog2e;
            ls = 0.0f;
        } else if (k < 10) {
            const int e = k - 2;
            pr[e] = exp2_fast(fmaf(x[e], kLog2e, nm));
            ls += pr[e];
        } else if (k == 10) {
            lrun += ls;
        }
    };
    auto s_mfma = [&](const char* tile, bf16x8_t* af, int k) __attribute__((always_inline)) {
        if constexpr (SP) {  // gap k: fragment k/2 = (k-step k/4, block (k/2)&1), token block k&1
            const int fa = k >> 1, mb = fa & 1, ks = fa >> 1;
            if (k & 1)
                so[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[fa], hf[KH + ks], so[mb], 0, 0, 0);
            else
                s[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[fa], hf[ks], s[mb], 0, 0, 0);
        } else {
            const int mb = k / KS, ks = k % KS;
            s[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k], hf[ks], s[mb], 0, 0, 0);
        }
    };
    // SP: W row fragment fa of a tile (rows 16(fa&1) + c, the half's k-step fa>>1)
    auto sp_frag = [&](const char* tile, int fa) __attribute__((always_inline)) {
        return ll16_row_frag(tile, rbh, fa & 1, fa >> 1);
    };
    auto sx_write = [&]() __attribute__((always_inline)) {
        *reinterpret_cast<f32x4_t*>(sxw) = so[0];
        *reinterpret_cast<f32x4_t*>(sxw + 1024) = so[1];
    };
#if LL_STAMP
    unsigned long long stamp[8] = {};
#endif
    // step t (t + 1 < t1): restrict LDS regions (alias scopes, as ll_fwd_block)
    auto step = [&](const char* __restrict__ cur, const char* __restrict__ nx, char* __restrict__ fut, int t)
                    __attribute__((always_inline)) {
        unsigned long long ts0 = 0, ts1 = 0, ts2 = 0, ts2b = 0, ts3 = 0;
        LL_TS(ts0);
        // this wave's pieces of tile t+1 (SAVEP: the previous step's P store, issued after
        // them, may still fly — it has this step to land)
        if (kFill == 2 && t > t0) {
            // the wave's own ds_writes of tile t+1 (the barrier's lgkmcnt); the P store may fly
        } else if (SAVEP && t > t0) {
            __builtin_amdgcn_s_waitcnt(ll_vmcnt(1));
        } else {
            __builtin_amdgcn_s_waitcnt(ll_vmcnt(0));
        }
        ll_lds_barrier();  // every wave's; every wave is done with tile t-1
        LL_TS(ts1);
        constexpr int PF = LL_FWD_PF;  // W row fragments in flight (LDS latency under a saturated array)
        bf16x8_t af[NG];
        f32x4_t xr[2];
        if constexpr (SP) {
            xr[0] = *reinterpret_cast<const f32x4_t*>(sxr);  // the partner's partial of S(t)
            xr[1] = *reinterpret_cast<const f32x4_t*>(sxr + 1024);
#pragma unroll
            for (int k = 0; k < PF; ++k) af[k] = sp_frag(nx, k);
        } else {
#pragma unroll
            for (int k = 0; k < PF; ++k) af[k] = ll16_row_frag(nx, rb, k / KS, k % KS);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e)  // S(t) for the softmax; S(t+1) accumulates anew
            x[e] = SP ? s[e >> 2][e & 3] + xr[e >> 2][e & 3] : s[e >> 2][e & 3];
        s[0] = f32x4_t{};
        s[1] = f32x4_t{};
        so[0] = f32x4_t{};
        so[1] = f32x4_t{};
        bf16x8_t pb;
        s16x8_t pt;
        vec4u ldv[NI];  // kFill 2: tile t+2's 16-B chunks of this lane
        bf16x8_t tfx[OF];  // OX: tile t's transposed fragments (the first PFX in the S loop's last gaps)
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            if (SP) {
                if (!(k & 1) && (k >> 1) + PF < KS) af[(k >> 1) + PF] = sp_frag(nx, (k >> 1) + PF);
            } else if (k + PF < NG) {
                af[k + PF] = ll16_row_frag(nx, rb, (k + PF) / KS, (k + PF) % KS);
            }
            s_mfma(nx, af, k);
            if (SAVEP && (!SP || PSL) && k == kPS) {
                if (kLLAblate & 64) {  // diagnostic: no LDS round trip (wrong layout)
                    pt = __builtin_bit_cast(s16x8_t, pb);
                } else {
                    pt = p_stage(pb);  // PSL: after the slot write at gap 12
                }
            }
            if (k == 0) {  // the lane's max + token max (no mask inside the loop: see ll_fwd_block)
                const float lm = fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])),
                                       fmaxf(fmaxf(x[4], x[5]), fmaxf(x[6], x[7])));
                m4 = ll_rows_max(lm);
            } else if (k == 2) {
                sm_chunk(1, t, std::false_type{});
            } else if (k >= 3 && k < 11) {
                sm_chunk(k - 1, t, std::false_type{});
            } else if (k == 11) {
                sm_chunk(10, t, std::false_type{});
                pb = pack8(pr);
            } else if (OX && k == 12) {
                *reinterpret_cast<bf16x8_t*>(xch) = pb;  // the exchange: read after the S loop's barrier
            }
            if (kFill == 0 && piece_at(k) && !(kLLAblate & 2048)) issue_piece(t + 2, fut, (k - kPO) / kPG);
            if (kFill == 2 && piece_at(k)) ldv[(k - kPO) / kPG] = load_piece(t + 2, (k - kPO) / kPG);
            if (OX && k >= NG - PFX) tfx[k - (NG - PFX)] = ox_frag(cur, k - (NG - PFX));
            __builtin_amdgcn_sched_barrier(0);
        }
        LL_TS(ts2);
        if constexpr (OX) {
            ll_lds_barrier();  // every wave's P(t) in the exchange
            LL_TS(ts2b);
            ox_product(cur, tfx, NG, [&](int gk) __attribute__((always_inline)) {
                const int f = gk - NG;
                // SP: P(t) through the transpose image, then S(t+1)'s partner partial into the
                // same region (the partner read the last one before the exchange barrier)
                if (SP && SAVEP && !PSL && f == 0) pt = ll_p_stage(pscr, pb, lane);
                if (SP && f == 1) sx_write();
                if (kFill == 1 && !(kLLAblate & 2048)) issue_piece(t + 2, fut, f);
                if (kFill == 2) *reinterpret_cast<vec4u*>(fut + (wave + G::kWaves * f) * 1024 + 16 * lane) = ldv[f];
            });
        } else {
        // ---- O(t): tr reads of tile t's W (cur) | MFMA
        constexpr int PFO = 4;
        bf16x8_t tf[DB];
#pragma unroll
        for (int nb = 0; nb < PFO; ++nb) tf[nb] = ll16_tr_frag(cur, trb, nb);
#pragma unroll
        for (int nb = 0; nb < DB; ++nb) {
            if (nb + PFO < DB) tf[nb + PFO] = ll16_tr_frag(cur, trb, nb + PFO);
            O[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tf[nb], pb, O[nb], 0, 0, 0);
            if (SAVEP && NG + nb == kPS) pt = ll_p_stage(pscr, pb, lane);
            const int gk = NG + nb;
            if (piece_at(gk)) issue_piece(t + 2, fut, (gk - kPO) / kPG);
            __builtin_amdgcn_sched_barrier(0);
        }
        }
        static_assert(kPG * (NI - 1) + kPO < NG + DB, "every DMA piece before the P store (the step's counted wait)");
        if (SAVEP && !(kLLAblate & 32)) ll_p_store(a, pt, t, ptt, phalf, lane);
        LL_TS(ts3);
#if LL_STAMP
        stamp[0] += ts1 - ts0;
        stamp[1] += ts2 - ts1;
        stamp[2] += ts3 - ts2;
        if (OX) stamp[3] += ts2b - ts2;
        stamp[6] += 1;
#endif
        (void)ts0, (void)ts1, (void)ts2, (void)ts2b, (void)ts3;
    };
    if (t0 < t1) {
        char* c0 = smem;
        char* c1 = smem + kStage;
        char* c2 = smem + 2 * kStage;
#pragma unroll
        for (int k = 0; k < NI; ++k) issue_piece(t0, c0, k);
#pragma unroll
        for (int k = 0; k < NI; ++k) issue_piece(t0 + 1, c1, k);
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(NI));  // tile t0 (t0+1 may fly)
        ll_lds_barrier();
        s[0] = f32x4_t{};
        s[1] = f32x4_t{};
        if constexpr (SP) {
            so[0] = f32x4_t{};
            so[1] = f32x4_t{};
#pragma unroll
            for (int fa = 0; fa < KS; ++fa) {
                const bf16x8_t f = sp_frag(c0, fa);
                s[fa & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f, hf[fa >> 1], s[fa & 1], 0, 0, 0);
                so[fa & 1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f, hf[KH + (fa >> 1)], so[fa & 1], 0, 0, 0);
            }
            sx_write();
        } else {
#pragma unroll
            for (int k = 0; k < NG; ++k) {
                const bf16x8_t af = ll16_row_frag(c0, rb, k / KS, k % KS);
                s[k / KS] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, hf[k % KS], s[k / KS], 0, 0, 0);
            }
        }
        for (int t = t0; t + 1 < t1; ++t) {
            step(c0, c1, c2, t);
            char* cc = c0;
            c0 = c1;
            c1 = c2;
            c2 = cc;
        }
        // the last tile: its (masked) softmax and O product
        if constexpr (SP) {
            ll_lds_barrier();  // the partner's partial of the last tile; every wave done with the P exchange
            s[0] += *reinterpret_cast<const f32x4_t*>(sxr);
            s[1] += *reinterpret_cast<const f32x4_t*>(sxr + 1024);
        }
#pragma unroll
        for (int k = 0; k < 11; ++k) sm_chunk(k, t1 - 1, std::true_type{});
        const bf16x8_t pb = pack8(pr);
        if constexpr (OX) {
            if (!SP) ll_lds_barrier();  // every wave is done reading the exchange of the previous tile
            *reinterpret_cast<bf16x8_t*>(xch) = pb;
            ll_lds_barrier();
            bf16x8_t tfx[OF];
#pragma unroll
            for (int f = 0; f < PFX; ++f) tfx[f] = ox_frag(c0, f);
            ox_product(c0, tfx, 0, [](int) {});
        } else {
#pragma unroll
            for (int nb = 0; nb < DB; ++nb)
                O[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ll16_tr_frag(c0, trb, nb), pb, O[nb], 0, 0, 0);
        }
        if (SAVEP) ll_p_store(a, p_stage(pb), t1 - 1, ptt, phalf, lane);
    }
#if LL_STAMP
    if (!RESTART && lane == 0 && lin * 4 + wave < (1 << 12))
        for (int k = 0; k < 8; ++k) g_ll_stamps[(lin * 4 + wave) * 8 + k] = stamp[k];
#endif
    // per-wave overflow flag (ll_fwd_block); the token's true max and Σ over its four lanes
    bool any = false;
    if (!RESTART) {
        any = __any(bad);
        if (lane == 0) a.flags[lin * G::kWaves + wave] = any;
    }
    const float mt4 = ll_rows_max(mtrue);
    const float mrun = any ? mt4 : mfix;
    const float lt = ll_rows_sum(lrun);
    if constexpr (OX) {
        // Oᵀ of token block tb, d = 16(16i + 4·wave + j) + 4g + r
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) {
            const int tmb = mt * kLLTokBlock + 16 * tb + c;
            if (tmb < nv) {
                float* op = a.opart + (int64_t(split) * a.N + tmb) * a.H + 64 * wave + 4 * g;
#pragma unroll
                for (int f = 0; f < OF; ++f)
                    *reinterpret_cast<f32x4_t*>(op + 256 * (f >> 2) + 16 * (f & 3)) = O[4 * f + tb];
            }
        }
        if (valid && g == 0) a.mlpart[int64_t(split) * a.N + tm] = make_float2(mrun, lt);
    } else if (valid) {
        float* op = a.opart + (int64_t(split) * a.N + tm) * a.H + 4 * g;
#pragma unroll
        for (int nb = 0; nb < DB; ++nb) *reinterpret_cast<f32x4_t*>(op + 16 * nb) = O[nb];
        if (g == 0) a.mlpart[int64_t(split) * a.N + tm] = make_float2(mrun, lt);
    }
}

// The first launch: one (token block, split) per workgroup; the split count follows the live
// token count (ll_fwd_splits), and each XCD (blockIdx % 8) takes a contiguous run of the
// split-major order, so the workgroups sharing an L2 stream the same W rows.  The RESTART
// launch (one workgroup per CU) walks the blocks and reruns the flagged ones.
template <class G, bool RESTART, bool F16, bool SAVEP = false>
__global__ __launch_bounds__(G::kThreads, 1) void k_lmloss_fwd(LmLossArgs a) {
    static_assert(F16 || !SAVEP, "the saved-P layout comes from the 16x16x32 form");
    __shared__ __attribute__((aligned(16))) char smem[3 * G::kStage + G::kWaves * 4096];
    static_assert(3 * G::kStage + G::kWaves * 4096 <= 163840, "forward LDS: 3 stages + exchange");
    const int nv = a.rows ? *a.nrows : a.N;
    const int ntb = (nv + 32 * G::NG - 1) / (32 * G::NG);
    const int nsplit = ll_fwd_splits(a, ntb);
    const int total = ntb * nsplit;
    if (!RESTART) {
        const int per_xcd = (total + 7) / 8;
        const int kx = int(blockIdx.x) >> 3, lin = (int(blockIdx.x) & 7) * per_xcd + kx;
        if (kx >= per_xcd || lin >= total) return;  // past an XCD's share / the live tokens
        if (F16)
            ll_fwd16_block<G, false, SAVEP>(a, smem, lin, ntb, nsplit, nv);
        else
            ll_fwd_block<G, false>(a, smem, lin, ntb, nsplit, nv);
        return;
    }
    for (int lin = int(blockIdx.x); lin < total; lin += int(gridDim.x)) {
        int f = 0;
#pragma unroll
        for (int w = 0; w < G::kWaves; ++w) f |= a.flags[lin * G::kWaves + w];
        if (!f) continue;
        if (F16)
            ll_fwd16_block<G, true, SAVEP>(a, smem, lin, ntb, nsplit, nv);
        else
            ll_fwd_block<G, true>(a, smem, lin, ntb, nsplit, nv);
        ll_lds_barrier();  // every wave is done with the LDS before the next block reuses it
    }
}

// ------------------------------------------------------------------ combine
// One workgroup per compact token m, one thread per 4 hidden columns (blockDim = H/4: 192 / 128):
// merge the vocab splits (fixed order), lse, lp, g, dh.  Every load a thread needs is issued
// before the one barrier (the cross-wave sum of the label logit): the splits' partial O and
// (m, l) first — they depend on m only, splits past nsplit re-read the last one and are weighted
// 0 — then the label row, and the PPO scalars, which every thread reads (same addresses) so
// that each computes g itself and no second barrier broadcasts it.
template <int MODE>
__global__ __launch_bounds__(256) void k_lmloss_combine(LmLossArgs a) {
    const int m = blockIdx.x, d4 = threadIdx.x;
    __shared__ float s_tok[4];
    int row = m;
    bool pad = false;
    const int nv = a.rows ? *a.nrows : a.N;
    if (a.rows) {
        const int r = a.rows[m];
        pad = m >= nv;
        row = pad ? ~r : r;
    }
    if (pad) {  // a masked token (mask == 0): zero gradient, no logits needed (masked_row)
        if (MODE == kLLPpo && d4 == 0) {
            float vin[3];
            const PpoScalars p = ppo_scalars(a, row, vin, true);
            PolicyTerms pt;
            ppo_policy_dlp(0.0f, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
            a.lp_out[row] = 0.0f;
            token_record(a, row, pt, p, vin);
            if (a.coef || a.wstats) split_outputs(a, row, p);
        }
        if (a.dh_dtype == TRLX_BF16)
            reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.dh) + int64_t(row) * a.lddh)[d4] = make_uint2(0u, 0u);
        else
            reinterpret_cast<f32x4_t*>(static_cast<float*>(a.dh) + int64_t(row) * a.lddh)[d4] = f32x4_t{};
        return;
    }
    const int H4 = a.H >> 2;
    f32x4_t op[kLLMaxSplits];
    float2 ml[kLLMaxSplits];
    int nsplit = 0;
    if (MODE != kLLBwd) {
        nsplit = ll_fwd_splits(a, (nv + kLLTokBlock - 1) / kLLTokBlock);
#pragma unroll
        for (int s = 0; s < kLLMaxSplits; ++s) {
            const int64_t sc = min(s, nsplit - 1);
            op[s] = reinterpret_cast<const f32x4_t*>(a.opart + (sc * a.N + m) * a.H)[d4];
            ml[s] = a.mlpart[sc * a.N + m];
        }
    }
    const int64_t y = a.labels[int64_t(row) * a.lb];
    const bool yok = y >= 0 && y < a.V;
    const uint2 wv = reinterpret_cast<const uint2*>(a.w + (yok ? y : 0) * a.ldw)[d4];
    float lse = 0.0f, L = 1.0f, g = 0.0f;
    f32x4_t e;
    if (MODE != kLLBwd) {
        const uint2 hv = reinterpret_cast<const uint2*>(a.h + int64_t(row) * a.ldh)[d4];
        float vin[3] = {0.0f, 0.0f, 0.0f};
        PpoScalars p{};
        if (MODE == kLLPpo) p = ppo_scalars(a, row, vin, true);
        // the label logit h·W[y] (fp32 products of the bf16 operands, fixed-order sums), kept
        // out of the forward's tile loop
        float xl = bf_lo(hv.x) * bf_lo(wv.x);
        xl = fmaf(bf_hi(hv.x), bf_hi(wv.x), xl);
        xl = fmaf(bf_lo(hv.y), bf_lo(wv.y), xl);
        xl = fmaf(bf_hi(hv.y), bf_hi(wv.y), xl);
        for (int off = 32; off > 0; off >>= 1) xl += __shfl_xor(xl, off);
        if ((d4 & 63) == 0) s_tok[d4 >> 6] = xl;
        __syncthreads();
        float xlab = s_tok[0];  // the waves' sums in wave order
        for (int w = 1; w < (H4 + 63) / 64; ++w) xlab += s_tok[w];
        float M = -INFINITY;
#pragma unroll
        for (int s = 0; s < kLLMaxSplits; ++s)
            if (s < nsplit) M = fmaxf(M, ml[s].x);
        L = 0.0f;
        e = f32x4_t{};
#pragma unroll
        for (int s = 0; s < kLLMaxSplits; ++s) {
            if (s >= nsplit) break;
            const float sc = ml[s].x == -INFINITY ? 0.0f : exp2_fast((ml[s].x - M) * kLog2e);
            L += ml[s].y * sc;
            e += sc * op[s];
        }
        const float lsum = logf(L);
        lse = M + lsum;
        e *= 1.0f / L;
        const float lp = yok ? (xlab - M) - lsum : NAN;  // the reference's order, as in the rows
        if (MODE == kLLPpo) {
            PolicyTerms pt;
            g = ppo_policy_dlp(lp, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
            if (a.prec && d4 < nsplit) {
                // the saved-P plan: split d4's record, dS = (y == v) ? g·(1 − p_y) : −g·e^(m_s − lse)·P
                float ms = ml[0].x;
#pragma unroll
                for (int s = 1; s < kLLMaxSplits; ++s) ms = d4 == s ? ml[s].x : ms;
                const float q = ms == -INFINITY ? 0.0f : g * exp2_fast((ms - lse) * kLog2e);
                const float dlab = fmaf(-g, exp2_fast(lp * kLog2e), g);
                a.prec[int64_t(d4) * a.N + m] = f32x4_t{q, dlab, __int_as_float(yok ? int(y) : -1), 0.0f};
            }
            if (d4 == 0) {
                const bool masked = p.m == 0.0f;
                a.lp_out[row] = masked ? 0.0f : lp;
                if (masked) ppo_policy_dlp(0.0f, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
                token_record(a, row, pt, p, vin);
                if (a.coef || a.wstats) split_outputs(a, row, p);
            }
        } else if (d4 == 0) {  // kLLFwd
            st_any(a.lp, a.lp_dtype, row, lp);
            if (a.lse_io) a.lse_io[row] = lse;
        }
    } else {  // kLLBwd: lse from the forward, g = the caller's d loss / d lp
        e = reinterpret_cast<const f32x4_t*>(a.ebuf + int64_t(row) * a.H)[d4];
        lse = a.lse_io[row];
        g = ld_any(a.gin, a.gin_dtype, row);
    }
    if (d4 == 0) {
        const f32x4_t rec = {-lse * kLog2e, g, __int_as_float(yok ? int(y) : -1), 0.0f};
        reinterpret_cast<f32x4_t*>(a.trec)[m] = rec;
    }
    if (MODE == kLLFwd) {
        reinterpret_cast<f32x4_t*>(a.ebuf + int64_t(row) * a.H)[d4] = e;
        return;
    }
    if (MODE == kLLBwd && !a.dh) return;  // hidden needs no gradient: the dW kernel's record only
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

// ------------------------------------------------------------------ dW
// Workgroup = 64 vocab rows x one token split, one wave per 16 rows holding them over the
// WHOLE hidden dimension (W fragments 96 registers, dW accumulators 192 at H = 768), so no
// partial S is ever exchanged between waves.  32-token tiles of h (+ their −lse·log2e, g, y)
// stream through LDS; per tile, on v_mfma_f32_16x16x32_bf16:
//   Sᵀ[t][v] = Σ_d h[t][d]·W[v][d]       2 token blocks x H/32 k-steps; h read by rows (A), the
//                                         W fragments the B operand: lane (g, c) ends with
//                                         tokens 16·mb + 4g + r of vocab row c
//   dS = g_t·(1[y_t = v] − 2^(S·log2e − lse_t·log2e))  — 8 tokens a lane, the scalars of 8 tokens
//   dW[v][d] += Σ_t dS[v][t]·h[t][d]     H/16 column blocks x ONE k-step of 32 tokens whose k
//                                         slots are permuted to what the lane holds: slot 8g + j
//                                         = token 4g + j (j < 4) / 16 + 4g + j − 4 — the A
//                                         operand is the lane's own 8 dS values, the B operand two
//                                         transposed reads (rows 4g.., 16 + 4g..) of the tile
// Twice the h bytes read from LDS per MFMA of the 32x32 pair form (each wave reads the whole
// tile, for S and for dW), in exchange for no group sum, no barrier inside the tile and the
// dS of one block computed beside the other block's MFMAs.
// Two forms measured slower at C2 (round 4, profiles/r04s_*): tiles staged through registers
// (buffer_load + ds_write_b128 instead of LDS-DMA: the dW phase 1,552 -> 2,018 cycles a tile)
// and a 3-stage software-pipelined step (dS(t) beside Sᵀ(t+1): the dS work moved, not hidden).
template <class G>
__global__ __launch_bounds__(256, 1) void k_lmloss_dw(LmLossArgs a) {
    constexpr int H = G::H, KS = H / 32, DB = H / 16, NI = G::NI;
    constexpr int kStage = G::kStage + 1024;  // h tile + the token records (16 B x 64 lanes)
    static_assert(G::kWaves == 4, "dW: four 16-row waves per 64-row workgroup");
    __shared__ __attribute__((aligned(16))) char smem[2 * kStage];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c = lane & 15;
    const int nv = a.rows ? *a.nrows : a.N;
    const int vpw = 64;
    // a whole vocab block over every token, or (the last round) a token split of one
    const bool part = int(blockIdx.x) >= a.dw_full;
    const int j = int(blockIdx.x) - a.dw_full;
    const int vb = part ? a.dw_full + j / a.tsplit : int(blockIdx.x);
    const int ts = part ? j % a.tsplit : 0, nts = part ? a.tsplit : 1;
    const int v0 = vb * vpw + wave * 16;  // this wave's 16 vocab rows
    const int vcol = v0 + c;
    const int ntt = (nv + kLLRows - 1) / kLLRows;
    const int t0 = int(int64_t(ts) * ntt / nts), t1 = int(int64_t(ts + 1) * ntt / nts);
    bf16x8_t wf[KS];  // B operand of Sᵀ: lane (g, c) -> W[v0 + c][32ks + 8g .. +7]
    if (vcol < a.V) {
        const uint16_t* wp = a.w + int64_t(vcol) * a.ldw + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[ks] = *reinterpret_cast<const bf16x8_t*>(wp + 32 * ks);
    } else {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) wf[ks] = bf16x8_t{};
    }
    // per-lane byte offsets in a staged tile (subtile image, ll_off):
    //   row read of token 16mb + c, columns 32ks + 8g: rb + 4096mb + (ks>>2)·8192 + (ks&3)·512
    //   transposed read of rows 4g + q (+16), columns 16nb + 4p: trb[nb&1] + (nb>>3)·8192 +
    //   ((nb&7)>>1)·512 (+4096)
    const int rb = ll16_rb(lane);
    const int trb[2] = {ll16_trb(lane, 0), ll16_trb(lane, 1)};
    auto row_frag = [&](const char* tile, int mb, int ks) __attribute__((always_inline)) {
        return ll16_row_frag(tile, rb, mb, ks);
    };
    auto tr_frag = [&](const char* tile, int nb) __attribute__((always_inline)) { return ll16_tr_frag(tile, trb, nb); };
    // the tile rows this lane's DMA pieces fetch (pieces i = wave + 4k: two distinct rows); row
    // N (out of the resource) past the live tokens: those rows are zero-filled, and so are their
    // records (g = 0, S = 0)
    auto tok_row = [&](int m) { return m < nv ? (a.rows ? a.rows[m] : m) : a.N; };
    int rowA = 0, rowB = 0, nrowA = 0, nrowB = 0;
    const int rA = ll_piece_row(wave, lane), rB = ll_piece_row(wave + G::kWaves, lane);
    if (t0 < t1) {
        rowA = tok_row(t0 * kLLRows + rA);
        rowB = tok_row(t0 * kLLRows + rB);
        nrowA = tok_row((t0 + 1) * kLLRows + rA);
        nrowB = tok_row((t0 + 1) * kLLRows + rB);
    }
    const __amdgpu_buffer_rsrc_t rh = make_rsrc(a.h, uint32_t(int64_t(a.N) * a.ldh * 2));
    const __amdgpu_buffer_rsrc_t rrec = make_rsrc(a.trec, uint32_t(a.N) * 16u);
    auto issue_piece = [&](int t, char* slot, int k, int ra, int rbw) __attribute__((always_inline)) {
        const int i = wave + G::kWaves * k;
        // 24-bit multiply (rows < 2^24, row bytes < 2^24): a 32-bit product here became a
        // v_mad_u64_u32 whose unused high addend register was a pending load's destination
        const int rbytes = int(__umul24(uint32_t(((i & 7) == (wave & 7)) ? ra : rbw), uint32_t(a.ldh) * 2u));
        const int off = ll16_piece_src(i, rbytes, lane);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rh, (__attribute__((address_space(3))) void*)(slot + i * 1024), 16,
                                                 t < t1 ? off : int(0x7ffff000), 0, 0, 0);
    };
    // the token records of tile t (wave 0): token t·32 + (l & 31)'s 16 B at byte 16·l (lanes l
    // and l+32 alike); zero past the live tokens — with their zero h rows, dS = 0 exactly
    // (S = 0, p = 2^0, g = 0) and no per-value test
    auto issue_scalars = [&](int t, char* slot) __attribute__((always_inline)) {
        const int m = t * kLLRows + (lane & 31);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rrec, (__attribute__((address_space(3))) void*)(slot + G::kStage),
                                                 16, t < t1 && m < nv ? m * 16 : int(0x7ffffff0), 0, 0, 0);
    };
    f32x4_t D[DB];  // dW[v0 + 4g + r][16nb + c]
#pragma unroll
    for (int nb = 0; nb < DB; ++nb) D[nb] = f32x4_t{};
    if (t0 < t1) {
#pragma unroll
        for (int k = 0; k < NI; ++k) issue_piece(t0, smem, k, rowA, rowB);
        if (wave == 0) issue_scalars(t0, smem);
    }
    constexpr int NG = 2 * KS;  // S-phase gaps
    // one tile; the LDS regions as __restrict__ parameters (alias scopes, as the forward)
    // tile t+2's rows: loaded unconditionally (a zero-size resource without compaction), picked
    // at the next tile — a load under a branch made hipcc wait for it at the branch's join
    const __amdgpu_buffer_rsrc_t rrows = make_rsrc(a.rows, a.rows ? uint32_t(a.N) * 4u : 0u);
#if LL_STAMP
    unsigned long long stamp[8] = {};
#endif
    auto tile = [&](const char* __restrict__ cur, char* __restrict__ nxt, int t) __attribute__((always_inline)) {
        unsigned long long ts1 = 0, ts2 = 0, ts3 = 0, ts4 = 0;
        LL_TS(ts1);
        const int ma = (t + 1) * kLLRows + rA, mb1 = (t + 1) * kLLRows + rB;  // tile t+1's rows
        const int pa = ma < nv ? (a.rows ? nrowA : ma) : a.N;
        const int pb = mb1 < nv ? (a.rows ? nrowB : mb1) : a.N;
        nrowA = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 2) * kLLRows + rA, nv - 1) * 4, 0, 0);
        nrowB = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 2) * kLLRows + rB, nv - 1) * 4, 0, 0);
        const char* scb = cur + G::kStage;
        f32x4_t snl[2], sgg[2];
        int4 syy[2];
        f32x4_t sacc[2] = {f32x4_t{}, f32x4_t{}};
        float ds[8];
        // dS = g·(1[y = v] − p) as g − g·p / −g·p (one fma; g = 0 past the live tokens)
        auto dsv = [&](int mb, int r) __attribute__((always_inline)) {
            const float gv = sgg[mb][r];
            const float pv = exp2_fast(fmaf(sacc[mb][r], kLog2e, snl[mb][r]));
            ds[4 * mb + r] = fmaf(-gv, pv, syy[mb][r] == vcol ? gv : 0.0f);
        };
        // ---- S phase: gap k = 24mb + ks (mb-major): row read k+PF | MFMA | DMA piece every
        // 4th gap | the tile's records read in gaps 2..9 | dS of block 0 in the gaps of block 1
        constexpr int PF = 4;
        bf16x8_t af[NG];
#pragma unroll
        for (int k = 0; k < PF; ++k) af[k] = row_frag(cur, k / KS, k % KS);
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            if (k + PF < NG) af[k + PF] = row_frag(cur, (k + PF) / KS, (k + PF) % KS);
            const int mb = k / KS, ks = k % KS;
            sacc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[k], wf[ks], sacc[mb], 0, 0, 0);
            if ((k & 3) == 1 && (k >> 2) < NI) issue_piece(t + 1, nxt, k >> 2, pa, pb);
            if (k >= 2 && k < 10) {  // token 16·b2 + 4g + r's record
                const int n = k - 2, b2 = n >> 2, r = n & 3;
                const f32x4_t rec = *reinterpret_cast<const f32x4_t*>(scb + 16 * (16 * b2 + 4 * g + r));
                snl[b2][r] = rec.x;
                sgg[b2][r] = rec.y;
                syy[b2][r] = __float_as_int(rec.z);
            }
            if (k >= KS + 4 && k < KS + 8) dsv(0, k - KS - 4);  // block 0's S is final (+latency)
            __builtin_amdgcn_sched_barrier(0);
        }
        LL_TS(ts2);
        if (wave == 0) issue_scalars(t + 1, nxt);
#pragma unroll
        for (int r = 0; r < 4; ++r) dsv(1, r);
        const bf16x8_t da = pack8(ds);  // A operand: slot 8g + j <- token t(g, j)
        __builtin_amdgcn_sched_barrier(0);
        LL_TS(ts3);
        // ---- dW phase: gap nb: tr reads nb+PFO | MFMA | the remaining DMA pieces
        constexpr int PFO = 4;
        bf16x8_t tf[DB];
#pragma unroll
        for (int nb = 0; nb < PFO; ++nb) tf[nb] = tr_frag(cur, nb);
#pragma unroll
        for (int nb = 0; nb < DB; ++nb) {
            if (nb + PFO < DB) tf[nb + PFO] = tr_frag(cur, nb + PFO);
            D[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, tf[nb], D[nb], 0, 0, 0);
            const int gk = NG + nb;  // global gap index
            if ((gk & 3) == 1 && (gk >> 2) < NI) issue_piece(t + 1, nxt, gk >> 2, pa, pb);
            __builtin_amdgcn_sched_barrier(0);
        }
        LL_TS(ts4);
#if LL_STAMP
        stamp[1] += ts2 - ts1;
        stamp[2] += ts3 - ts2;
        stamp[3] += ts4 - ts3;
        stamp[6] += 1;
#endif
        (void)ts1, (void)ts2, (void)ts3, (void)ts4;
    };
    for (int t = t0; t < t1; ++t) {
        unsigned long long ts0 = 0, ts1 = 0;
        LL_TS(ts0);
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(0));  // this wave's pieces of tile t
        ll_lds_barrier();  // every wave's; and every wave is done with tile t-1
        LL_TS(ts1);
#if LL_STAMP
        stamp[0] += ts1 - ts0;
#endif
        (void)ts0, (void)ts1;
        tile(smem + ((t - t0) & 1) * kStage, smem + ((t + 1 - t0) & 1) * kStage, t);
    }
#if LL_STAMP
    if (lane == 0 && blockIdx.x * 4 + wave < (1 << 12))
        for (int k = 0; k < 8; ++k) g_ll_stamps[(1 << 15) + (blockIdx.x * 4 + wave) * 8 + k] = stamp[k];
#endif
    // D[nb][r] = dW(vocab v0 + 4g + r, hidden 16nb + c)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int vr = wave * 16 + 4 * g + r, v = vb * vpw + vr;
        if (part) {  // fp32 partial of this token split, summed by k_lmloss_dw_reduce
            float* out = a.dwpart + (int64_t(j) * vpw + vr) * H + c;
#pragma unroll
            for (int nb = 0; nb < DB; ++nb) out[16 * nb] = D[nb][r];
        } else if (v < a.V) {
            const int64_t o = int64_t(v) * a.lddw + c;
            if (a.dw_dtype == TRLX_F32) {
                float* out = static_cast<float*>(a.dw) + o;
#pragma unroll
                for (int nb = 0; nb < DB; ++nb) out[16 * nb] = D[nb][r];
            } else {
                uint16_t* out = static_cast<uint16_t*>(a.dw) + o;
#pragma unroll
                for (int nb = 0; nb < DB; ++nb) out[16 * nb] = f2bf(D[nb][r]);
            }
        }
    }
}

// ------------------------------------------------------------------ dW from the saved P
// k_lmloss_dw without its Sᵀ pass: the forward left every bf16 P tile in HBM in this kernel's
// A-operand layout (ll_p_stage / ll_p_store) and the combine a record per (split, token)
// {q = g·e^(m_split − lse), dlab = g·(1 − p_y), y}, so dS = (y == v) ? dlab : −q·P — the P of the
// E product rescaled to the final lse, the label entry from the fp32 label logit.  Workgroup =
// 64·RW vocab rows (4 waves x 16·RW rows over the whole H; dW accumulators 192·RW registers at
// H = 768) x one token split; per 32-token tile ONE product, dW += dS·h_tile (RW x H/16 MFMAs
// v_mfma_f32_16x16x32_bf16; the h tile read transposed, each fragment feeding RW MFMAs: lane
// group g's k slots = tokens 8g..8g+7, rows 8g + q and 8g + 4 + q of the subtile image —
// conflict-free on the ll16_swz image).  RW = 2 halves the h bytes staged and read from LDS per
// MFMA (the RW = 1 form's dW phase ran at ~2.7x its MFMA time, bound by the DMA issue and the
// LDS reads).  The dS of the NEXT tile is formed in the MFMA gaps (records read in two groups
// of 4, the values after them).  Loads run ahead: a 3-stage h ring (the DMA of tile t+2 during
// tile t), 3 record slots (tile t+3), P chunks in 3 register sets (tile t+3's load issued at
// tile t), and the barrier waits only for what was issued before the previous tile (counted
// vmcnt: P streams from HBM, 0.62 GB per call at C2).
#ifndef LL_DWP_PFO
#define LL_DWP_PFO 8  // transposed h fragments in flight
#endif
#ifndef LL_DWP_PIECE_GAP
#define LL_DWP_PIECE_GAP 4
#endif
#ifndef LL_DWP_PIECE_OFF
#define LL_DWP_PIECE_OFF 1
#endif
template <class G, int RW, int HSP>
__global__ __launch_bounds__(256, 1) void k_lmloss_dwp(LmLossArgs a) {
    // HSP = 2: a workgroup owns HALF the hidden columns of its vocab rows (h part hp = blockIdx
    // & 1, the two parts of a block adjacent in dispatch order so the second P read hits the
    // Infinity Cache): RW = 2 then holds 32 rows x H/2 = 192 accumulators, the RW = 1 budget
    constexpr int H = G::H, HC = H / HSP, DB = HC / 16, NI = G::NI / HSP;
    constexpr int kStage = G::kStage / HSP;
    constexpr int kRecSlot = RW == 1 ? 1024 : 4096;  // RW = 2: each wave's own 1-KB records
    static_assert(G::kWaves == 4, "dW: four waves per workgroup");
    static_assert(HC % 128 == 0, "h parts of whole 128-column segments");
    static_assert(3 * kStage + 3 * kRecSlot <= 163840, "3 h stages + 3 record slots");
    // the next-but-one tile's h pieces every kPG-th gap from kPO on
    constexpr int kPG = LL_DWP_PIECE_GAP, kPO = LL_DWP_PIECE_OFF;
    static_assert(kPO < kPG && kPG * (NI - 1) + kPO < DB, "every DMA piece inside the tile's gaps");
    // + each wave's RW KB of dS hand-off (below)
    static_assert(3 * kStage + 3 * kRecSlot + 4096 * RW <= 163840, "LDS budget with the dS hand-off");
    __shared__ __attribute__((aligned(16))) char smem[3 * kStage + 3 * kRecSlot + 4096 * RW];
    char* recs = smem + 3 * kStage;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    char* dsl = recs + 3 * kRecSlot + 1024 * RW * wave + 16 * lane;
    const int g = lane >> 4, c = lane & 15, q = (lane >> 2) & 3, p = lane & 3;
    const int nv = a.rows ? *a.nrows : a.N;
    constexpr int vpw = 64 * RW;
    const int hp = HSP == 1 ? 0 : int(blockIdx.x) & 1, bid = int(blockIdx.x) / HSP;
    const bool part = bid >= a.dw_full;
    const int j = bid - a.dw_full;
    const int vb = part ? a.dw_full + j / a.tsplit : bid;
    const int ts = part ? j % a.tsplit : 0, nts = part ? a.tsplit : 1;
    const int r0 = vb * vpw + wave * 16 * RW;  // this wave's first vocab row
    const int ntt = (nv + kLLRows - 1) / kLLRows;
    const int t0 = int(int64_t(ts) * ntt / nts), t1 = int(int64_t(ts + 1) * ntt / nts);
    // the forward's split of the vocab tiles (ll_fwd_splits: the same plan)
    const int nsplit = ll_fwd_splits(a, (nv + kLLTokBlock - 1) / kLLTokBlock);
    const int nvt = (a.V + kLLRows - 1) / kLLRows;
    auto split_of = [&](int vt) {
        int s = 0;
        for (int k = 1; k < nsplit; ++k) s = int(int64_t(k) * nvt / nsplit) <= vt ? k : s;
        return s;
    };
    // the records this lane DMAs and where the wave reads its tokens' records (+ 16·j)
    const int srec = RW == 1 ? split_of(2 * vb + (lane >> 5)) : split_of(4 * vb + wave);
    const int rdst = RW == 1 ? 0 : 1024 * wave;
    const int rb16 = (RW == 1 ? 512 * (wave >> 1) : 1024 * wave) + 16 * (8 * g);
    // transposed reads of the h tile: rows 8g + 4hf + q, columns 16nb + 4p (ll_off image)
    int trb8[2][2];
#pragma unroll
    for (int par = 0; par < 2; ++par)
#pragma unroll
        for (int hf = 0; hf < 2; ++hf)
            trb8[par][hf] = 2048 * g + 64 * (4 * hf + q) + 16 * ((2 * par + (p >> 1)) ^ ll16_swz((2 * g + hf) & 3)) +
                            8 * (p & 1);
    auto tr_frag = [&](const char* tile, int nb) __attribute__((always_inline)) {
        typedef __attribute__((address_space(3))) s16x4_t lds_s4;
        const int off = (nb >> 3) * 8192 + ((nb & 7) >> 1) * 512;
        const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(tile + trb8[nb & 1][0] + off));
        const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(tile + trb8[nb & 1][1] + off));
        const s16x8_t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        return __builtin_bit_cast(bf16x8_t, v);
    };
    auto tok_row = [&](int m) { return m < nv ? (a.rows ? a.rows[m] : m) : a.N; };
    const int rA = ll_piece_row(wave, lane), rB = ll_piece_row(wave + G::kWaves, lane);
    const __amdgpu_buffer_rsrc_t rh = make_rsrc(a.h, uint32_t(int64_t(a.N) * a.ldh * 2));
    const __amdgpu_buffer_rsrc_t rrec = make_rsrc(a.prec, uint32_t(kLLMaxSplits) * uint32_t(a.N) * 16u);
    const __amdgpu_buffer_rsrc_t rrows = make_rsrc(a.rows, a.rows ? uint32_t(a.N) * 4u : 0u);
    auto stage = [&](int t) __attribute__((always_inline)) { return smem + (t % 3) * kStage; };
    auto rslot = [&](int t) __attribute__((always_inline)) { return recs + (t % 3) * kRecSlot; };
    // piece il of the part's image = piece hp·HC/16 + il of the full-H image (a multiple of 8:
    // the same rows)
    auto issue_piece = [&](int t, char* slot, int k, int ra, int rbw) __attribute__((always_inline)) {
        const int il = wave + G::kWaves * k, i = hp * (HC / 16) + il;
        const int rbytes = int(__umul24(uint32_t(((il & 7) == (wave & 7)) ? ra : rbw), uint32_t(a.ldh) * 2u));
        const int off = ll16_piece_src(i, rbytes, lane);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rh, (__attribute__((address_space(3))) void*)(slot + il * 1024), 16,
                                                 t < t1 ? off : int(0x7ffff000), 0, 0, 0);
    };
    // records of tile t: lane l -> split srec, token t·32 + (l & 31), at byte rdst + 16·l of the
    // slot (RW = 1: lanes 32-63 the block's second vocab tile, every wave the same DMA; RW = 2:
    // each wave its own tile's, lanes 32-63 a copy); zero past the live tokens (q = dlab = 0:
    // dS = 0 whatever P holds there).  No wave-dependent branch: every wave's count of loads in
    // flight is the same and the counted waits stay exact.
    auto issue_recs = [&](int t, char* slot) __attribute__((always_inline)) {
        const int m = t * kLLRows + (lane & 31);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rrec, (__attribute__((address_space(3))) void*)(slot + rdst), 16,
                                                 t < t1 && m < nv ? (srec * a.N + m) * 16 : int(0x7ffffff0), 0, 0,
                                                 0);
    };
    // P chunk of tile t for row half hh (rows r0 + 16hh + c, tokens 8g..8g+7), clamped to the
    // split's last tile: 64-row block (r0 + 16hh) / 64, dW wave slot ((r0 + 16hh) / 16) & 3
    const s16x8_t* pbase[RW];
#pragma unroll
    for (int hh = 0; hh < RW; ++hh) {
        const int rr0 = r0 + 16 * hh;
        pbase[hh] = reinterpret_cast<const s16x8_t*>(a.pbuf) + (int64_t(rr0 >> 6) * a.pntt * 4 + ((rr0 >> 4) & 3)) * 64 +
                    lane;
    }
    auto load_p = [&](int t, int hh) __attribute__((always_inline)) {
        return pbase[hh][int64_t(min(t, t1 - 1)) * 256];
    };
    auto ds_of = [&](const f32x4_t& rec, short pe, int vcol) __attribute__((always_inline)) {
        const float pv = __uint_as_float(uint32_t(uint16_t(pe)) << 16);
        return __float_as_int(rec.z) == vcol ? rec.y : -rec.x * pv;
    };
    auto rec_at = [&](const char* slot, int e) __attribute__((always_inline)) {
        return *reinterpret_cast<const f32x4_t*>(slot + rb16 + 16 * e);
    };
    f32x4_t D[RW][DB];  // dW[r0 + 16hh + 4g + r][16nb + c]
#pragma unroll
    for (int hh = 0; hh < RW; ++hh)
#pragma unroll
        for (int nb = 0; nb < DB; ++nb) D[hh][nb] = f32x4_t{};
    bf16x8_t da[RW];
    s16x8_t R0[RW], R1[RW], R2[RW];  // P(t0 + k) in R[k % 3]
#pragma unroll
    for (int hh = 0; hh < RW; ++hh) {
        da[hh] = bf16x8_t{};
        R0[hh] = R1[hh] = R2[hh] = s16x8_t{};
    }
    int nrowA = 0, nrowB = 0;  // rows of tile t+2 at the start of tile t
    if (t0 < t1) {
        const int rowA0 = tok_row(t0 * kLLRows + rA), rowB0 = tok_row(t0 * kLLRows + rB);
        const int rowA1 = tok_row((t0 + 1) * kLLRows + rA), rowB1 = tok_row((t0 + 1) * kLLRows + rB);
        nrowA = a.rows ? a.rows[min((t0 + 2) * kLLRows + rA, nv - 1)] : 0;
        nrowB = a.rows ? a.rows[min((t0 + 2) * kLLRows + rB, nv - 1)] : 0;
#pragma unroll
        for (int hh = 0; hh < RW; ++hh) {
            R0[hh] = load_p(t0, hh);
            R1[hh] = load_p(t0 + 1, hh);
            R2[hh] = load_p(t0 + 2, hh);
        }
#pragma unroll
        for (int k = 0; k < NI; ++k) issue_piece(t0, stage(t0), k, rowA0, rowB0);
#pragma unroll
        for (int k = 0; k < NI; ++k) issue_piece(t0 + 1, stage(t0 + 1), k, rowA1, rowB1);
        issue_recs(t0, rslot(t0));
        issue_recs(t0 + 1, rslot(t0 + 1));
        issue_recs(t0 + 2, rslot(t0 + 2));
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(0));
        ll_lds_barrier();
#pragma unroll
        for (int hh = 0; hh < RW; ++hh) {
            float ds[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) ds[e] = ds_of(rec_at(rslot(t0), e), R0[hh][e], r0 + 16 * hh + c);
            da[hh] = pack8(ds);
        }
    }
#if LL_STAMP
    unsigned long long stamp[8] = {};
#endif
    // tile t: dW(t) with da = dS(t); in its gaps the loads of the tiles ahead and dS(t+1) from
    // puse = P(t+1) and the records of t+1 (rnx); pnew receives P(t+3).  The LDS regions are
    // __restrict__ parameters (alias scopes: the DMA targets fut / rfut apart from the regions
    // read, as k_lmloss_dw — without them hipcc waits for the DMA before every read).
    auto tile_body = [&](const char* __restrict__ cur, char* __restrict__ fut, const char* __restrict__ rnx,
                         char* __restrict__ rfut, int t, const s16x8_t (&puse)[RW], s16x8_t (&pnew)[RW])
                         __attribute__((always_inline)) {
        const int ma = (t + 2) * kLLRows + rA, mb1 = (t + 2) * kLLRows + rB;  // tile t+2's rows
        const int pa = ma < nv ? (a.rows ? nrowA : ma) : a.N;
        const int pb = mb1 < nv ? (a.rows ? nrowB : mb1) : a.N;
        nrowA = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 3) * kLLRows + rA, nv - 1) * 4, 0, 0);
        nrowB = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 3) * kLLRows + rB, nv - 1) * 4, 0, 0);
        if (!(kLLAblate & 128)) {
#pragma unroll
            for (int hh = 0; hh < RW; ++hh) pnew[hh] = load_p(t + 3, hh);
        }
        bf16x8_t dn[RW];
        f32x4_t rr[8];
        float dsn[RW][8];
        // gaps: the 8 records read at kR (4 + 4), then one dS value per gap from kD on (L gaps
        // ≈ 128 MFMA cycles later; one at a time, so the VALU work hides behind the MFMAs of
        // its gap: four values in one gap had cost ~400 cycles a tile), the packs after them;
        // transposed reads PFO fragments ahead (≈ 256 MFMA cycles)
        constexpr int PFO = LL_DWP_PFO, L = 8 / RW, kR = 1, kD = kR + 1 + L;
        constexpr int VPG = (8 * RW + (DB - kD - 2)) / (DB - kD - 1);  // dS values per gap
        constexpr int kPk = kD + (8 * RW + VPG - 1) / VPG;
        static_assert(kPk < DB, "the dS gaps");
        bf16x8_t tf[DB];
#pragma unroll
        for (int nb = 0; nb < PFO; ++nb) tf[nb] = tr_frag(cur, nb);
#pragma unroll
        for (int nb = 0; nb < DB; ++nb) {
            if (nb + PFO < DB) tf[nb + PFO] = tr_frag(cur, nb + PFO);
#pragma unroll
            for (int hh = 0; hh < RW; ++hh)
                D[hh][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[hh], tf[nb], D[hh][nb], 0, 0, 0);
            // (the four waves' pieces in the same gaps: staggering them by wave — a wave-uniform
            // branch per gap — measured slower in both kernels, the forward's S loop 2,033 ->
            // 3,900 cycles a tile)
            if (nb % kPG == kPO && nb / kPG < NI && !(kLLAblate & 256)) issue_piece(t + 2, fut, nb / kPG, pa, pb);
            if (nb == 2) issue_recs(t + 3, rfut);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (nb == kR) rr[e] = rec_at(rnx, e);
                if (nb == kR + 1) rr[4 + e] = rec_at(rnx, 4 + e);
            }
#pragma unroll
            for (int hh = 0; hh < RW; ++hh) {
#pragma unroll
                for (int e = 0; e < 8; ++e)
                    if (nb == kD + (RW * e + hh) / VPG) {
                        dsn[hh][e] = ds_of(rr[e], puse[hh][e], r0 + 16 * hh + c);
                        asm volatile("" : "+v"(dsn[hh][e]));  // formed in this gap, not sunk to the store
                    }
                // the next tile's A operand goes through the wave's LDS slot and is read back after
                // this tile's last MFMA: handed over in registers (dn copied into da), hipcc gave
                // both the same registers and sank the whole dS computation to after the last
                // MFMA (~400 cycles a tile, serial; ISA); the store pins it to its gaps
                if (nb == kPk) {
                    *reinterpret_cast<bf16x8_t*>(dsl + 1024 * hh) = pack8(dsn[hh]);
                    asm volatile("" ::: "memory");
                }
            }
            if (nb == DB - 1) {
                asm volatile("" ::: "memory");
#pragma unroll
                for (int hh = 0; hh < RW; ++hh) dn[hh] = *reinterpret_cast<const bf16x8_t*>(dsl + 1024 * hh);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if (!(kLLAblate & 512)) {
#pragma unroll
            for (int hh = 0; hh < RW; ++hh) da[hh] = dn[hh];
        }
    };
    auto tile = [&](int t, const s16x8_t (&puse)[RW], s16x8_t (&pnew)[RW]) __attribute__((always_inline)) {
        unsigned long long ts0 = 0, ts1 = 0, ts2 = 0;
        LL_TS(ts0);
        // everything issued before the previous tile (2 row indices, RW P chunks, NI pieces, the
        // records: NI + 3 + RW per tile): h(t), the records and P of t+1
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(NI + 3 + RW));
        ll_lds_barrier();
        LL_TS(ts1);
        tile_body(stage(t), stage(t + 2), rslot(t + 1), rslot(t + 3), t, puse, pnew);
        LL_TS(ts2);
#if LL_STAMP
        stamp[0] += ts1 - ts0;
        stamp[3] += ts2 - ts1;
        stamp[6] += 1;
#endif
        (void)ts0, (void)ts1, (void)ts2;
    };
    for (int t = t0; t < t1; t += 3) {
        tile(t, R1, R0);
        if (t + 1 < t1) tile(t + 1, R2, R1);
        if (t + 2 < t1) tile(t + 2, R0, R2);
    }
#if LL_STAMP
    if (lane == 0 && blockIdx.x * 4 + wave < (1 << 12))
        for (int k = 0; k < 8; ++k) g_ll_stamps[(1 << 15) + (blockIdx.x * 4 + wave) * 8 + k] = stamp[k];
#endif
#pragma unroll
    for (int hh = 0; hh < RW; ++hh)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int vr = wave * 16 * RW + 16 * hh + 4 * g + r, v = vb * vpw + vr;
            if (part) {
                float* out = a.dwpart + (int64_t(j) * vpw + vr) * H + hp * HC + c;
#pragma unroll
                for (int nb = 0; nb < DB; ++nb) out[16 * nb] = D[hh][nb][r];
            } else if (v < a.V) {
                const int64_t o = int64_t(v) * a.lddw + hp * HC + c;
                if (a.dw_dtype == TRLX_F32) {
                    float* out = static_cast<float*>(a.dw) + o;
#pragma unroll
                    for (int nb = 0; nb < DB; ++nb) out[16 * nb] = D[hh][nb][r];
                } else {
                    uint16_t* out = static_cast<uint16_t*>(a.dw) + o;
#pragma unroll
                    for (int nb = 0; nb < DB; ++nb) out[16 * nb] = f2bf(D[hh][nb][r]);
                }
            }
        }
}

// Fixed-order sum of the token-split dW partials of the vocab blocks past dw_full:
// dw[v][d] = Σ_ts part[b·tsplit + ts][r][d] for v = (dw_full + b)·vpw + r.
__global__ __launch_bounds__(256) void k_lmloss_dw_reduce(const float* part, int tsplit, int nblk, int dw_full,
                                                          int vpw, void* dw, int dw_dtype, int V, int H,
                                                          int64_t lddw) {
    const int64_t per4 = int64_t(vpw) * H / 4, n4 = nblk * per4;  // 4 columns a thread (H % 4 == 0)
    for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n4; i += int64_t(gridDim.x) * blockDim.x) {
        const int64_t b = i / per4, e = i - b * per4, r = (4 * e) / H, d = 4 * e - r * H;
        const int64_t v = (dw_full + b) * vpw + r;
        if (v >= V) continue;
        const f32x4_t* src = reinterpret_cast<const f32x4_t*>(part) + b * tsplit * per4 + e;
        f32x4_t acc = src[0];
        for (int s = 1; s < tsplit; ++s) acc += src[s * per4];
#pragma unroll
        for (int c = 0; c < 4; ++c) st_any(dw, dw_dtype, v * lddw + d + c, acc[c]);
    }
}

// ------------------------------------------------------------------ H-sliced forms (round 5)
// Both MFMA kernels as ONE engine whose four waves split the hidden dimension instead of the
// rows: wave q owns hidden columns [q·HS, (q+1)·HS), HS = H/4, for its register operand (64
// rows x HS: 96 registers at H = 768) AND its accumulators (64 rows x HS fp32: 192), and the
// workgroup streams 16-row tiles of the other operand through a 4-slot LDS ring:
//   dW:      registers = W rows v0..v0+63,  tiles = h (16 tokens),  accumulators = dWᵀ
//   forward: registers = h rows m0..m0+63,  tiles = W (16 vocab),   accumulators = Oᵀ
// Per tile: the partial S over the wave's slice (16x16x32: M = the 16 tile rows, N = 4 blocks
// of 16 register rows, K = 32 hidden columns — every row fragment read from LDS feeds 4 MFMAs),
// the four partials summed through LDS by the wave that owns register block q (fixed order
// w = 0..3), its X step — dS = g·(1[y = v] − p) (dW) or P = exp(S − offset) (forward) — into a
// bf16 [64 register rows][16 tile rows] image, and the second product (32x32x16: M = 32 hidden
// columns, N = 32 register rows, K = the 16 tile rows; the tile read transposed, each fragment
// feeding 2 MFMAs).  Against the row-split forms (k_lmloss_dw: a wave per 16 vocab rows over
// the whole H, every tile fragment feeding ONE MFMA) this reads a quarter of the tile bytes
// from LDS per MFMA, which was the dW kernel's bound.
// The step is pipelined three tiles deep with ONE barrier per tile:
//   phase t:  MFMA S(t) [rows of tile t] + MFMA P(t-2) [tile t-2 transposed, X(t-2)]
//             VALU X(t-1) [partials of S(t-1) -> X image]; writes S(t) partials; DMA tile t+1
// so a phase's barrier publishes S(t-1)'s partials, X(t-2)'s image and tile t's bytes at
// once.  LDS: 4 tile slots (24 KB at H = 768, + 1 KB of token records for dW), 2 partial
// buffers (16 KB: [writer][block][lane] f32x4), 2 X images (2 KB) = 136 KB.
// Tile image: two 8-row groups of [8 rows][H] in 512-B subtiles (8 rows x 32 columns), the
// 16-B chunk slot XOR-swizzled by ll16_swz((row>>2)&3): conflict-free for the 16x16x32 row
// reads and the 32x32x16 transposed reads (MI355X_MICROARCH.md LDS banking), and every read of
// a wave is one of three lane bases plus an immediate (512 B per 32-column group).
template <int H_>
struct HsG {
    static constexpr int H = H_, HS = H / 4, KS = HS / 32, CB = HS / 32;
    static constexpr int kRows = 16, kTile = kRows * H * 2;
    static constexpr int kPieces = kTile / 1024, NI = kPieces / 4, NPR = H / 64;
    static constexpr int kRowGroup = 8 * H * 2;
    static constexpr int kSlot = kTile + 1024;
    static constexpr int kXBuf = 16 * 1024;
    static constexpr int kXs = 64 * 32;
    static constexpr int kLds = 4 * kSlot + 2 * kXBuf + 2 * kXs;
    static_assert(kPieces % 4 == 0 && NI == KS && kLds <= 163840, "H-sliced geometry");
};

// the tile row lane `lane` of DMA piece i fills, and its source chunk (16 B units of the row)
template <class G>
__device__ __forceinline__ int hs_piece_row(int i, int lane) {
    return 8 * (i / G::NPR) + ((lane >> 2) & 7);
}
template <class G>
__device__ __forceinline__ int hs_piece_chunk(int i, int lane) {
    const int r = hs_piece_row<G>(i, lane);
    const int u = 2 * (i % G::NPR) + (lane >> 5);
    return 4 * u + ((lane & 3) ^ ll16_swz((r >> 2) & 3));
}
// lane bases: row read (16x16x32 operand: tile row lane&15, chunk 4u + (lane>>4)) and the two
// halves of a transposed read (32x32x16 operand: column lane&31 of a 32-column group, tile
// rows 8(lane>>5) + 4·half + 0..3)
template <class G>
__device__ __forceinline__ int hs_rb(int lane) {
    const int g = lane >> 4, c = lane & 15;
    return (c >> 3) * G::kRowGroup + 64 * (c & 7) + 16 * (g ^ ll16_swz((c >> 2) & 3));
}
template <class G>
__device__ __forceinline__ int hs_trb(int lane, int half) {
    const int G4 = lane >> 4, qq = (lane >> 2) & 3, p = lane & 3;
    const int r = 8 * (G4 >> 1) + 4 * half + qq;
    return (G4 >> 1) * G::kRowGroup + 64 * (r & 7) + 16 * ((2 * (G4 & 1) + (p >> 1)) ^ ll16_swz((r >> 2) & 3)) +
           8 * (p & 1);
}
__device__ __forceinline__ bf16x8_t hs_row(const char* tile, int rb, int u) {
    return *reinterpret_cast<const bf16x8_t*>(tile + rb + 512 * u);
}
__device__ __forceinline__ bf16x8_t hs_tr(const char* tile, int trb0, int trb1, int u) {
    typedef __attribute__((address_space(3))) s16x4_t lds_s4;
    const s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(tile + trb0 + 512 * u));
    const s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(tile + trb1 + 512 * u));
    const s16x8_t v = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    return __builtin_bit_cast(bf16x8_t, v);
}
// X image [64 register rows][16 tile rows] bf16, 32 B a row, the 16-B halves swapped on rows
// with bit 3 set: the B-operand read (row 32b + lane&31, tile rows 8(lane>>5)..+7) is
// conflict-free.
__device__ __forceinline__ int hs_xs_rd(int lane) {
    const int r = lane & 31;
    return r * 32 + 16 * ((lane >> 5) ^ ((r >> 3) & 1));
}
__device__ __forceinline__ int hs_xs_wr(int q, int g, int c) {
    return (16 * q + c) * 32 + 16 * ((g >> 1) ^ ((c >> 3) & 1)) + 8 * (g & 1);
}

enum { kHsDw = 0, kHsFwd = 1 };

// One 1-KB LDS-DMA piece as an asm statement (cdna_hip_programming.md §5.7: M0 written and
// restored inside it): hipcc does not model it, so it inserts no wait for the LDS reads still
// in flight when a piece is issued (the builtin form drew an lgkmcnt wait for every older
// ds_read before each piece: the compiler cannot tell the landing slot from the slots being
// read) — the engine waits for its own pieces with vmcnt(0) at the next phase.
__device__ __forceinline__ void hs_dma(__amdgpu_buffer_rsrc_t rs, const char* lds, int voff) {
    const uint32_t dst = __builtin_amdgcn_readfirstlane(
        uint32_t(uintptr_t((const __attribute__((address_space(3))) char*)lds)));
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
                 "s_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(voff), "s"(dst), "s"(rs)
                 : "memory");
}

// The engine.  ROLE kHsDw: rop = W fragments, the grid / token split of k_lmloss_dw; the
// caller stores acc2 as dWᵀ rows.  ROLE kHsFwd: rop = h fragments of token block m0, the vocab
// tiles [t0, t1) of one split; fixed exponent offset per token = its first tile's max
// (overflow -> the RESTART launch, as ll_fwd_block).  Returns through acc2 (+ the forward's
// per-token state in fs).
struct HsFwdState {
    float mfix, mtrue, lrun;
    bool bad;
};

template <class G, int ROLE, bool RESTART>
__device__ __forceinline__ void hs_engine(const LmLossArgs& a, char* smem, const bf16x8_t (&rop)[4][G::KS],
                                          f32x16_t (&acc2)[2][G::CB], int t0, int t1, int q, int v0, int nv,
                                          HsFwdState& fs) {
    constexpr int KS = G::KS, CB = G::CB, NI = G::NI;
    const int lane = threadIdx.x & 63;
    const int g = lane >> 4, c = lane & 15;
    const int u0 = q * (G::HS / 32);  // the wave's first 32-column group
    char* slots = smem;
    char* xbuf = smem + 4 * G::kSlot;
    char* xsb = xbuf + 2 * G::kXBuf;
    const int rb = hs_rb<G>(lane), trb0 = hs_trb<G>(lane, 0), trb1 = hs_trb<G>(lane, 1);
    const int xsr = hs_xs_rd(lane), xsw = hs_xs_wr(q, g, c);
    // ---- DMA sources
    const __amdgpu_buffer_rsrc_t rsrc =
        ROLE == kHsDw ? make_rsrc(a.h, uint32_t(int64_t(a.N) * a.ldh * 2)) : make_rsrc(a.w, uint32_t(int64_t(a.V) * a.ldw * 2));
    const int ld2 = ROLE == kHsDw ? int(a.ldh) * 2 : int(a.ldw) * 2;
    const __amdgpu_buffer_rsrc_t rrec = make_rsrc(a.trec, uint32_t(a.N) * 16u);
    const __amdgpu_buffer_rsrc_t rrows = make_rsrc(a.rows, a.rows ? uint32_t(a.N) * 4u : 0u);
    // dW: a lane's two source rows (tile rows (l>>2)&7 and 8 + that) of the next tile, by index
    // loads one tile ahead (compacted tokens); past the live tokens row N (zero fill)
    const int rA = (lane >> 2) & 7;
    auto tok_row = [&](int m) __attribute__((always_inline)) { return m < nv ? (a.rows ? a.rows[m] : m) : a.N; };
    int nrowA = 0, nrowB = 0;  // dW, compacted: the row indices of tile t+1, loaded during phase t-1
    auto piece = [&](int t, char* slot, int k, int rowa, int rowb) __attribute__((always_inline)) {
        const int i = q + 4 * k;
        const int r = hs_piece_row<G>(i, lane);
        int rbytes;
        if (ROLE == kHsDw)
            rbytes = int(__umul24(uint32_t(r < 8 ? rowa : rowb), uint32_t(ld2)));
        else
            rbytes = (t * 16 + r) * ld2;
        const int off = rbytes + 16 * hs_piece_chunk<G>(i, lane);
        hs_dma(rsrc, slot + i * 1024, t < t1 ? off : int(0x7ffff000));
    };
    auto records = [&](int t, char* slot) __attribute__((always_inline)) {  // dW: 16 tokens' {-lse·log2e, g, y}
        const int m = t * 16 + (lane & 15);
        hs_dma(rrec, slot + G::kTile, t < t1 && m < nv ? m * 16 : int(0x7ffffff0));
    };
    f32x4_t acc[4];
#if LL_STAMP
    unsigned long long hst[4] = {};  // steady phases: wait + barrier, S part, P part, count
    unsigned long long hts0 = 0, hts1 = 0;
#endif
    // ---- one phase (FL bit 1: S(t), 2: X(t-1), 4: P(t-2)); LDS regions as restrict parameters
    auto body = [&](auto fl_tag, int t, const char* __restrict__ cur, const char* __restrict__ old,
                    const char* __restrict__ prv, char* __restrict__ nxt, char* __restrict__ xw,
                    const char* __restrict__ xr, char* __restrict__ xsw_p, const char* __restrict__ xsr_p)
                    __attribute__((always_inline)) {
        constexpr int FL = decltype(fl_tag)::value;
        constexpr bool DS = FL & 1, DX = FL & 2, DP = FL & 4;
        constexpr int NGS = DS ? 4 * KS : 0, NGP = DP ? 2 * CB : 0, NG = NGS + NGP;
        // dW: this phase's DMA takes tile t+1's rows (row N past the live tokens: zero fill);
        // the index loads fetch tile t+2's (unconditional, picked next phase: a load under a
        // branch made hipcc wait for it at the join)
        int pa = 0, pb = 0;
        if (ROLE == kHsDw && DS) {
            const int ma = (t + 1) * 16 + rA, mb = ma + 8;
            pa = ma < nv ? (a.rows ? nrowA : ma) : a.N;
            pb = mb < nv ? (a.rows ? nrowB : mb) : a.N;
            nrowA = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 2) * 16 + rA, nv - 1) * 4, 0, 0);
            nrowB = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 2) * 16 + 8 + rA, nv - 1) * 4, 0, 0);
        }
        // LDS reads in the order of first use (LDS returns in order: a read waits for every
        // older one): S(t)'s first row fragments, X(t-2)'s operand, S(t-1)'s partials, records
        constexpr int PF = 3;
        bf16x8_t rf[KS];
        if (DS) {
#pragma unroll
            for (int ks = 0; ks < PF && ks < KS; ++ks) rf[ks] = hs_row(cur, rb, u0 + ks);
#pragma unroll
            for (int b = 0; b < 4; ++b) acc[b] = f32x4_t{};
        }
        bf16x8_t xsf[2];
        if (DP) {
            xsf[0] = *reinterpret_cast<const bf16x8_t*>(xsr_p + xsr);
            xsf[1] = *reinterpret_cast<const bf16x8_t*>(xsr_p + xsr + 1024);
        }
        f32x4_t xv[4];
        f32x4_t rec[4];
        if (DX) {
#pragma unroll
            for (int w = 0; w < 4; ++w) xv[w] = reinterpret_cast<const f32x4_t*>(xr + (w * 4 + q) * 1024)[lane];
            if (ROLE == kHsDw) {
#pragma unroll
                for (int r = 0; r < 4; ++r) rec[r] = *reinterpret_cast<const f32x4_t*>(prv + G::kTile + 16 * (4 * g + r));
            }
        }
        bf16x8_t tf[CB];
        float s[4], xo[4];
        // X chunks: 0 sum, 1 (fwd) token max, 2 offset, 3 exp + pack (dW: 1 exp + dS, 2 pack)
        // X(t-1) in eight micro-steps of at most ~5 vector instructions (one transcendental
        // pair), one per MFMA gap of the P part (32-cycle gaps leave ~24 cycles of issue each;
        // MI355X_MICROARCH.md 'vector-instruction ISSUE cost'), the image store in the last.
        auto xmicro = [&](int m) __attribute__((always_inline)) {
            if (kLLAblate & 1) return;
            const int tp = t - 1;
            if (m < 2) {
#pragma unroll
                for (int r = 2 * m; r < 2 * m + 2; ++r) s[r] = ((xv[0][r] + xv[1][r]) + xv[2][r]) + xv[3][r];
                return;
            }
            if (ROLE == kHsDw) {
                if (m == 2 || m == 3) {
#pragma unroll
                    for (int r = 2 * (m - 2); r < 2 * (m - 2) + 2; ++r) {
                        asm volatile("" ::"v"(rec[r]));  // the whole 16-B record live until here: no WAW
                                                         // stall on its unused word
                        xo[r] = exp2_fast(fmaf(s[r], kLog2e, rec[r].x));
                    }
                } else if (m == 4 || m == 5) {
                    const int vcol = v0 + 16 * q + c;
#pragma unroll
                    for (int r = 2 * (m - 4); r < 2 * (m - 4) + 2; ++r) {
                        const float gv = rec[r].y;
                        xo[r] = fmaf(-gv, xo[r], __float_as_int(rec[r].z) == vcol ? gv : 0.0f);
                    }
                } else if (m == 6) {
                    *reinterpret_cast<uint2*>(xsw_p + xsw) = make_uint2(pack_bf2(xo[0], xo[1]), pack_bf2(xo[2], xo[3]));
                }
            } else {
                if (m == 2) {
                    if ((tp + 1) * 16 > a.V) {  // the vocab's last tile (wave-uniform): rows past V
                        const int lim = a.V - tp * 16 - 4 * g;
#pragma unroll
                        for (int r = 0; r < 4; ++r) s[r] = r < lim ? s[r] : -INFINITY;
                    }
                    xo[0] = fmaxf(fmaxf(s[0], s[1]), fmaxf(s[2], s[3]));
                } else if (m == 3) {
                    const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(xo[0]), __float_as_uint(xo[0]),
                                                                     false, false);
                    xo[0] = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));  // lanes l, l^16
                } else if (m == 4) {
                    const float mx = ll_pair_max(xo[0]);  // lanes l, l^32: the token's 16 tile rows
                    if (!RESTART) {
                        fs.mtrue = fmaxf(fs.mtrue, mx);
                        fs.mfix = tp == t0 ? mx : fs.mfix;
                        fs.bad = fs.bad || mx > fs.mfix + kLLOverflow;
                    }
                    xo[1] = -fs.mfix * kLog2e;
                } else if (m == 5 || m == 6) {
                    const float nm = xo[1];
#pragma unroll
                    for (int r = 2 * (m - 5); r < 2 * (m - 5) + 2; ++r) s[r] = exp2_fast(fmaf(s[r], kLog2e, nm));
                } else if (m == 7) {
                    fs.lrun += (s[0] + s[1]) + (s[2] + s[3]);
                    *reinterpret_cast<uint2*>(xsw_p + xsw) = make_uint2(pack_bf2(s[0], s[1]), pack_bf2(s[2], s[3]));
                }
            }
        };
        constexpr int NXM = 8;
        // where micro-step m runs: P gap XJ0 + m; without a P part, the last 8 S gaps; without
        // either, straight after the loop
        constexpr int XJ0 = 2 * CB >= NXM + 1 ? 1 : 0;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            if (k < NGS) {
                const int ks = k >> 2, b = k & 3;
                if (b == 0 && ks + PF < KS) rf[ks + PF] = hs_row(cur, rb, u0 + ks + PF);
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rf[ks], rop[b][ks], acc[b], 0, 0, 0);
                if ((k & 3) == 1 && (k >> 2) < NI && !(kLLAblate & 4)) {
                    piece(t + 1, nxt, k >> 2, pa, pb);
                    if (ROLE == kHsDw && q == 0 && (k >> 2) == 0) records(t + 1, nxt);
                }
                if (DP && k >= NGS - 6 && ((NGS - k) & 1) == 0 && (NGS - k) / 2 <= 3)  // tf[0..2], 2 gaps apart
                    tf[3 - (NGS - k) / 2] = hs_tr(old, trb0, trb1, u0 + 3 - (NGS - k) / 2);
            } else if (k < NG) {
                const int j = k - NGS, cb = j >> 1, b2 = j & 1;
                if (!DS && j == 0) {
#pragma unroll
                    for (int x = 0; x < 3 && x < CB; ++x) tf[x] = hs_tr(old, trb0, trb1, u0 + x);
                }
                if (b2 == 0 && cb + 3 < CB) tf[cb + 3] = hs_tr(old, trb0, trb1, u0 + cb + 3);
                acc2[b2][cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf[cb], xsf[b2], acc2[b2][cb], 0, 0, 0);
                if (DS && j >= 1 && j <= 4)  // S(t)'s partials (their MFMAs done)
                    reinterpret_cast<f32x4_t*>(xw + (q * 4 + (j - 1)) * 1024)[lane] = acc[j - 1];
            }
            if (DX) {
                constexpr int XK0 = DP ? NGS + XJ0 : NGS - NXM;
#pragma unroll
                for (int m = 0; m < NXM; ++m)
                    if (k == XK0 + m) xmicro(m);
            }
            __builtin_amdgcn_sched_barrier(0);
#if LL_STAMP
            if (FL == 7 && k == NGS - 1) {
                unsigned long long tsx = 0;
                LL_TS(tsx);
                hst[1] += tsx - hts1;
                hts1 = tsx;
            }
#endif
        }
#if LL_STAMP
        if (FL == 7) {
            unsigned long long tsx = 0;
            LL_TS(tsx);
            hst[2] += tsx - hts1;
            hst[3] += 1;
        }
#endif
        if (DS && !DP) {  // no P MFMAs to carry them: S(t)'s partials now
#pragma unroll
            for (int b = 0; b < 4; ++b) reinterpret_cast<f32x4_t*>(xw + (q * 4 + b) * 1024)[lane] = acc[b];
        }
        if (DX && NG == 0) {
#pragma unroll
            for (int m = 0; m < NXM; ++m) xmicro(m);
        }
    };
    auto phase = [&](auto fl_tag, int t) __attribute__((always_inline)) {
#if LL_STAMP
        LL_TS(hts0);
#endif
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(0));  // this wave's pieces of tile t (and the index loads)
        ll_lds_barrier();                          // everyone's: tile t, S(t-1) partials, X(t-2)
#if LL_STAMP
        LL_TS(hts1);
        if (decltype(fl_tag)::value == 7) hst[0] += hts1 - hts0;
#endif
        body(fl_tag, t, slots + (t & 3) * G::kSlot, slots + ((t - 2) & 3) * G::kSlot,
             slots + ((t - 1) & 3) * G::kSlot, slots + ((t + 1) & 3) * G::kSlot, xbuf + (t & 1) * G::kXBuf,
             xbuf + ((t - 1) & 1) * G::kXBuf, xsb + ((t - 1) & 1) * G::kXs, xsb + ((t - 2) & 1) * G::kXs);
    };
    if (t0 >= t1) return;
    {  // prologue: tile t0's DMA
        char* s0 = slots + (t0 & 3) * G::kSlot;
        const int ra0 = ROLE == kHsDw ? tok_row(t0 * 16 + rA) : 0, rb0 = ROLE == kHsDw ? tok_row(t0 * 16 + 8 + rA) : 0;
#pragma unroll
        for (int k = 0; k < NI; ++k) piece(t0, s0, k, ra0, rb0);
        if (ROLE == kHsDw && q == 0) records(t0, s0);
        if (ROLE == kHsDw && a.rows) {  // tile t0+1's row indices
            nrowA = a.rows[min((t0 + 1) * 16 + rA, nv - 1)];
            nrowB = a.rows[min((t0 + 1) * 16 + 8 + rA, nv - 1)];
        }
    }
    using F1 = std::integral_constant<int, 1>;
    using F3 = std::integral_constant<int, 3>;
    using F7 = std::integral_constant<int, 7>;
    using F6 = std::integral_constant<int, 6>;
    using F2 = std::integral_constant<int, 2>;
    using F4 = std::integral_constant<int, 4>;
    phase(F1{}, t0);
    if (t0 + 1 < t1) {
        phase(F3{}, t0 + 1);
        for (int t = t0 + 2; t < t1; ++t) phase(F7{}, t);
        phase(F6{}, t1);
    } else {
        phase(F2{}, t1);
    }
    phase(F4{}, t1 + 1);
#if LL_STAMP
    {  // per wave: fwd at [0, 2^15), dW at [2^15, 2^16) of g_ll_stamps, 8 words a wave
        const int slot = int(blockIdx.x) * 4 + q;
        if (lane == 0 && slot < (1 << 12))
            for (int k = 0; k < 4; ++k) g_ll_stamps[(ROLE == kHsDw ? (1 << 15) : 0) + slot * 8 + k] = hst[k];
    }
#endif
}

// dW, H-sliced: per 64-row vocab block (or, in the last partial round, a token split of one:
// the plan of k_lmloss_dw), the engine over the block's 16-token tiles of h, then dWᵀ rows:
// lane l holds vocab row v0 + 32b + (l&31) at 16 columns in runs of 4 (f32x4 / 8-B stores).
template <class G>
__global__ __launch_bounds__(256, 1) void k_lmloss_dw_hs(LmLossArgs a) {
    constexpr int KS = G::KS, CB = G::CB, HS = G::HS;
    __shared__ __attribute__((aligned(16))) char smem[G::kLds];
    const int lane = threadIdx.x & 63;
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, c = lane & 15;
    const int nv = a.rows ? *a.nrows : a.N;
    const bool part = int(blockIdx.x) >= a.dw_full;
    const int j = int(blockIdx.x) - a.dw_full;
    const int vb = part ? a.dw_full + j / a.tsplit : int(blockIdx.x);
    const int ts = part ? j % a.tsplit : 0, nts = part ? a.tsplit : 1;
    const int v0 = vb * 64;
    const int ntt = (nv + 15) / 16;
    const int t0 = int(int64_t(ts) * ntt / nts), t1 = int(int64_t(ts + 1) * ntt / nts);
    bf16x8_t wf[4][KS];  // B operand of S: W[v0 + 16b + c][q·HS + 32ks + 8g .. +7]
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int v = v0 + 16 * b + c;
        const uint16_t* wp = a.w + int64_t(v < a.V ? v : 0) * a.ldw + q * HS + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            wf[b][ks] = v < a.V ? *reinterpret_cast<const bf16x8_t*>(wp + 32 * ks) : bf16x8_t{};
    }
    f32x16_t acc2[2][CB];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc2[b][cb] = f32x16_t{};
    HsFwdState fs{};
    hs_engine<G, kHsDw, false>(a, smem, wf, acc2, t0, t1, q, v0, nv, fs);
    // acc2[b][cb][r] = dW[v0 + 32b + (l&31)][q·HS + 32cb + 8(r>>2) + 4(l>>5) + (r&3)]
    const int hi = lane >> 5;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int vr = 32 * b + (lane & 31), v = v0 + vr;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4) {
                const int col = q * HS + 32 * cb + 8 * r4 + 4 * hi;
                const f32x4_t d = {acc2[b][cb][4 * r4], acc2[b][cb][4 * r4 + 1], acc2[b][cb][4 * r4 + 2],
                                   acc2[b][cb][4 * r4 + 3]};
                if (part) {  // fp32 partial of this token split (k_lmloss_dw_reduce)
                    *reinterpret_cast<f32x4_t*>(a.dwpart + (int64_t(j) * 64 + vr) * a.H + col) = d;
                } else if (v < a.V) {
                    const int64_t o = int64_t(v) * a.lddw + col;
                    if (a.dw_dtype == TRLX_F32)
                        *reinterpret_cast<f32x4_t*>(static_cast<float*>(a.dw) + o) = d;
                    else
                        *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.dw) + o) =
                            make_uint2(pack_bf2(d.x, d.y), pack_bf2(d.z, d.w));
                }
            }
    }
}

// Forward, H-sliced: per (64-token block, vocab split) the engine over the split's 16-row W
// tiles; Oᵀ: lane l holds token m0 + 32b + (l&31) at 16 columns in runs of 4; the owner of
// token block q (16 tokens) holds their (max, Σ) state.
template <class G, bool RESTART>
__device__ __forceinline__ void hs_fwd_block(const LmLossArgs& a, char* smem, int lin, int ntb, int nsplit, int nv) {
    constexpr int KS = G::KS, CB = G::CB, HS = G::HS;
    const int lane = threadIdx.x & 63;
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int g = lane >> 4, c = lane & 15;
    const int split = lin / ntb, mt = lin - split * ntb;
    const int m0 = mt * kLLTokBlock;
    bf16x8_t hf[4][KS];  // B operand of S: h[token m0 + 16b + c][q·HS + 32ks + 8g .. +7]
#pragma unroll
    for (int b = 0; b < 4; ++b) {
        const int tm = m0 + 16 * b + c, tc = tm < nv ? tm : nv - 1;
        const int row = a.rows ? a.rows[tc] : tc;
        const uint16_t* hp = a.h + int64_t(row) * a.ldh + q * HS + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) hf[b][ks] = *reinterpret_cast<const bf16x8_t*>(hp + 32 * ks);
    }
    const int nvt = (a.V + 15) / 16;
    const int t0 = int(int64_t(split) * nvt / nsplit), t1 = int(int64_t(split + 1) * nvt / nsplit);
    const int town = m0 + 16 * q + c;  // the token whose softmax state this lane carries
    const bool vown = town < nv;
    HsFwdState fs;
    fs.mfix = -INFINITY;
    fs.mtrue = -INFINITY;
    fs.lrun = 0.0f;
    fs.bad = false;
    if (RESTART) fs.mfix = a.mlpart[int64_t(split) * a.N + (vown ? town : nv - 1)].x;
    f32x16_t acc2[2][CB];
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int cb = 0; cb < CB; ++cb) acc2[b][cb] = f32x16_t{};
    hs_engine<G, kHsFwd, RESTART>(a, smem, hf, acc2, t0, t1, q, 0, nv, fs);
    bool any = false;
    if (!RESTART) {
        any = __any(fs.bad);
        if (lane == 0) a.flags[lin * 4 + q] = any;
    }
    const float mrun = any ? fs.mtrue : fs.mfix;
    float lt = fs.lrun + __shfl_xor(fs.lrun, 16);
    lt = lt + __shfl_xor(lt, 32);
    if (vown && g == 0) a.mlpart[int64_t(split) * a.N + town] = make_float2(mrun, lt);
    const int hi = lane >> 5;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int tm = m0 + 32 * b + (lane & 31);
        if (tm < nv) {
            float* op = a.opart + (int64_t(split) * a.N + tm) * a.H + q * HS + 4 * hi;
#pragma unroll
            for (int cb = 0; cb < CB; ++cb)
#pragma unroll
                for (int r4 = 0; r4 < 4; ++r4)
                    *reinterpret_cast<f32x4_t*>(op + 32 * cb + 8 * r4) =
                        f32x4_t{acc2[b][cb][4 * r4], acc2[b][cb][4 * r4 + 1], acc2[b][cb][4 * r4 + 2],
                                acc2[b][cb][4 * r4 + 3]};
        }
    }
}

template <class G, bool RESTART>
__global__ __launch_bounds__(256, 1) void k_lmloss_fwd_hs(LmLossArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[G::kLds];
    const int nv = a.rows ? *a.nrows : a.N;
    const int ntb = (nv + kLLTokBlock - 1) / kLLTokBlock;
    const int nsplit = ll_fwd_splits(a, ntb);
    const int total = ntb * nsplit;
    if (!RESTART) {
        const int per_xcd = (total + 7) / 8;
        const int kx = int(blockIdx.x) >> 3, lin = (int(blockIdx.x) & 7) * per_xcd + kx;
        if (kx >= per_xcd || lin >= total) return;
        hs_fwd_block<G, false>(a, smem, lin, ntb, nsplit, nv);
        return;
    }
    for (int lin = int(blockIdx.x); lin < total; lin += int(gridDim.x)) {
        int f = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) f |= a.flags[lin * 4 + w];
        if (!f) continue;
        hs_fwd_block<G, true>(a, smem, lin, ntb, nsplit, nv);
        ll_lds_barrier();
    }
}

// ------------------------------------------------------------------ H-sliced, two waves per SIMD
// The same engine with 8 waves (512 threads, <= 256 registers each): wave w = (group grp =
// w >> 2, slice q = w & 3) owns register rows 32·grp .. +31 over hidden slice q — 48 operand and
// 96 accumulator registers at H = 768 — so each SIMD holds one wave of each group, and one
// wave's stalls (LDS-DMA issue, X-step vector work, LDS waits) sit beside its partner's MFMAs
// (MI355X_MICROARCH.md 'Two waves per SIMD').  Per tile and wave: S 2 blocks x KS k-steps of
// 16x16x32, the group's partials summed by owner q (register rows 8q .. 8q+7 of the group, all
// 16 tile rows: 2 values a lane), P CB blocks of 32x32x16.  LDS as the 4-wave engine (the
// partial buffers: [group][writer][block][lane] f32x4, 16 KB).
template <int H_>
struct Hs8G {
    static constexpr int H = H_, HS = H / 4, KS = HS / 32, CB = HS / 32;
    static constexpr int kRows = 16, kTile = kRows * H * 2;
    static constexpr int kPieces = kTile / 1024, NI = kPieces / 8, NPR = H / 64;
    static constexpr int kRowGroup = 8 * H * 2;
    static constexpr int kRing = 5;            // tile slots: 2 tiles of DMA in flight
    static constexpr int kSlot = kTile + 256;  // + 16 token records (dW)
    static constexpr int kXBuf = 16 * 1024;
    static constexpr int kXs = 64 * 32;
    static constexpr int kLds = kRing * kSlot + 2 * kXBuf + 2 * kXs;
    static_assert(kPieces % 8 == 0 && kLds <= 163840, "8-wave H-sliced geometry");
};

template <class G, int ROLE, bool RESTART>
__device__ __forceinline__ void hs8_engine(const LmLossArgs& a, char* smem, const bf16x8_t (&rop)[2][G::KS],
                                           f32x16_t (&acc2)[G::CB], int t0, int t1, int w, int v0, int nv,
                                           HsFwdState& fs) {
    constexpr int KS = G::KS, CB = G::CB, NI = G::NI;
    const int lane = threadIdx.x & 63;
    const int grp = w >> 2, q = w & 3;
    const int u0 = q * (G::HS / 32);
    char* slots = smem;
    char* xbuf = smem + G::kRing * G::kSlot;
    char* xsb = xbuf + 2 * G::kXBuf;
    const int rb = hs_rb<G>(lane), trb0 = hs_trb<G>(lane, 0), trb1 = hs_trb<G>(lane, 1);
    const int xsr = (32 * grp + (lane & 31)) * 32 + 16 * ((lane >> 5) ^ (((lane & 31) >> 3) & 1));
    // the owner view: register row R8 = 8q + (lane & 7) of the group (block ob = q >> 1, column
    // oc = 8(q&1) + (lane&7) of its 16x16 partials), tile rows 2j, 2j+1 with j = lane >> 3
    const int j8 = lane >> 3, oc = 8 * (q & 1) + (lane & 7), ob = q >> 1;
    const int xoff = ob * 1024 + ((j8 >> 1) * 16 + oc) * 16 + 8 * (j8 & 1);  // in a writer's 2 KB
    const int xrow = 32 * grp + 16 * ob + oc;                               // X image row
    const int xsw = xrow * 32 + 16 * ((j8 >> 2) ^ ((xrow >> 3) & 1)) + 4 * (j8 & 3);
    const __amdgpu_buffer_rsrc_t rsrc =
        ROLE == kHsDw ? make_rsrc(a.h, uint32_t(int64_t(a.N) * a.ldh * 2)) : make_rsrc(a.w, uint32_t(int64_t(a.V) * a.ldw * 2));
    const int ld2 = ROLE == kHsDw ? int(a.ldh) * 2 : int(a.ldw) * 2;
    const __amdgpu_buffer_rsrc_t rrec = make_rsrc(a.trec, uint32_t(a.N) * 16u);
    const __amdgpu_buffer_rsrc_t rrows = make_rsrc(a.rows, a.rows ? uint32_t(a.N) * 4u : 0u);
    const int rA = (lane >> 2) & 7;
    auto tok_row = [&](int m) __attribute__((always_inline)) { return m < nv ? (a.rows ? a.rows[m] : m) : a.N; };
    int nrowA = 0, nrowB = 0;
    auto piece = [&](int t, char* slot, int k, int rowa, int rowb) __attribute__((always_inline)) {
        const int i = w + 8 * k;
        const int r = hs_piece_row<G>(i, lane);
        int rbytes;
        if (ROLE == kHsDw)
            rbytes = int(__umul24(uint32_t(r < 8 ? rowa : rowb), uint32_t(ld2)));
        else
            rbytes = (t * 16 + r) * ld2;
        const int off = rbytes + 16 * hs_piece_chunk<G>(i, lane);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (__attribute__((address_space(3))) void*)(slot + i * 1024), 16,
                                                 t < t1 ? off : int(0x7ffff000), 0, 0, 0);
    };
    auto records = [&](int t, char* slot) __attribute__((always_inline)) {  // lanes 0..15: 256 B
        const int m = t * 16 + lane;
        if (lane < 16)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rrec, (__attribute__((address_space(3))) void*)(slot + G::kTile),
                                                     16, t < t1 && m < nv ? m * 16 : int(0x7ffffff0), 0, 0, 0);
    };
    // DMA ops a wave issues per tile (its pieces + wave 0's records): the phase-start wait leaves
    // the younger tile's in flight
    const bool recw = ROLE == kHsDw && w == 0;
    auto slot_of = [&](int t) __attribute__((always_inline)) { return slots + ((t + 2 * G::kRing) % G::kRing) * G::kSlot; };
    f32x4_t acc[2];
#if LL_STAMP
    unsigned long long hst[4] = {};
    unsigned long long hts0 = 0, hts1 = 0;
#endif
    auto body = [&](auto fl_tag, int t, const char* __restrict__ cur, const char* __restrict__ old,
                    const char* __restrict__ prv, char* __restrict__ nxt, char* __restrict__ xw,
                    const char* __restrict__ xr, char* __restrict__ xsw_p, const char* __restrict__ xsr_p)
                    __attribute__((always_inline)) {
        constexpr int FL = decltype(fl_tag)::value;
        constexpr bool DS = FL & 1, DX = FL & 2, DP = FL & 4;
        constexpr int NGS = DS ? 2 * KS : 0, NGP = DP ? CB : 0, NG = NGS + NGP;
        int pa = 0, pb = 0;  // dW: tile t+2's source rows; the index loads fetch tile t+3's
        if (ROLE == kHsDw && DS) {
            const int ma = (t + 2) * 16 + rA, mb = ma + 8;
            pa = ma < nv ? (a.rows ? nrowA : ma) : a.N;
            pb = mb < nv ? (a.rows ? nrowB : mb) : a.N;
            nrowA = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 3) * 16 + rA, nv - 1) * 4, 0, 0);
            nrowB = __builtin_amdgcn_raw_buffer_load_b32(rrows, min((t + 3) * 16 + 8 + rA, nv - 1) * 4, 0, 0);
        }
        constexpr int PF = 2;
        bf16x8_t rf[KS];
        if (DS) {
#pragma unroll
            for (int ks = 0; ks < PF && ks < KS; ++ks) rf[ks] = hs_row(cur, rb, u0 + ks);
            acc[0] = f32x4_t{};
            acc[1] = f32x4_t{};
        }
        bf16x8_t xsf = bf16x8_t{};
        if (DP) xsf = *reinterpret_cast<const bf16x8_t*>(xsr_p + xsr);
        float2 xv[4];
        f32x4_t rec[2];
        if (DX) {
#pragma unroll
            for (int wq = 0; wq < 4; ++wq)
                xv[wq] = *reinterpret_cast<const float2*>(xr + ((grp * 4 + wq) * 2) * 1024 + xoff);
            if (ROLE == kHsDw) {
#pragma unroll
                for (int r = 0; r < 2; ++r) rec[r] = *reinterpret_cast<const f32x4_t*>(prv + G::kTile + 16 * (2 * j8 + r));
            }
        }
        bf16x8_t tf[CB];
        float s[2], xo[2];
        auto xmicro = [&](int m) __attribute__((always_inline)) {
            if (kLLAblate & 1) return;
            const int tp = t - 1;
            if (m == 0) {
                s[0] = ((xv[0].x + xv[1].x) + xv[2].x) + xv[3].x;
                s[1] = ((xv[0].y + xv[1].y) + xv[2].y) + xv[3].y;
                return;
            }
            if (ROLE == kHsDw) {
                if (m == 1) {
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        asm volatile("" ::"v"(rec[r]));
                        xo[r] = exp2_fast(fmaf(s[r], kLog2e, rec[r].x));
                    }
                } else if (m == 2) {
                    const int vcol = v0 + xrow;
#pragma unroll
                    for (int r = 0; r < 2; ++r) {
                        const float gv = rec[r].y;
                        xo[r] = fmaf(-gv, xo[r], __float_as_int(rec[r].z) == vcol ? gv : 0.0f);
                    }
                } else if (m == 3) {
                    *reinterpret_cast<uint32_t*>(xsw_p + xsw) = pack_bf2(xo[0], xo[1]);
                }
            } else {
                if (m == 1) {
                    if ((tp + 1) * 16 > a.V) {  // the vocab's last tile (wave-uniform): rows past V
                        const int lim = a.V - tp * 16 - 2 * j8;
                        s[0] = 0 < lim ? s[0] : -INFINITY;
                        s[1] = 1 < lim ? s[1] : -INFINITY;
                    }
                    xo[0] = fmaxf(s[0], s[1]);
                    // lanes l, l^8 (DPP row_ror:8 within a 16-lane row)
                    xo[0] = fmaxf(xo[0], __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(
                                             0, __builtin_bit_cast(int, xo[0]), 0x128, 0xf, 0xf, false)));
                } else if (m == 2) {
                    const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(xo[0]), __float_as_uint(xo[0]),
                                                                     false, false);
                    xo[0] = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));  // l, l^16
                    const float mx = ll_pair_max(xo[0]);                           // l, l^32
                    if (!RESTART) {
                        fs.mtrue = fmaxf(fs.mtrue, mx);
                        fs.mfix = tp == t0 ? mx : fs.mfix;
                        fs.bad = fs.bad || mx > fs.mfix + kLLOverflow;
                    }
                    xo[1] = -fs.mfix * kLog2e;
                } else if (m == 3) {
                    s[0] = exp2_fast(fmaf(s[0], kLog2e, xo[1]));
                    s[1] = exp2_fast(fmaf(s[1], kLog2e, xo[1]));
                    fs.lrun += s[0] + s[1];
                    *reinterpret_cast<uint32_t*>(xsw_p + xsw) = pack_bf2(s[0], s[1]);
                }
            }
        };
        constexpr int NXM = 4;
#pragma unroll
        for (int k = 0; k < NG; ++k) {
            if (k < NGS) {
                const int ks = k >> 1, b = k & 1;
                if (b == 0 && ks + PF < KS) rf[ks + PF] = hs_row(cur, rb, u0 + ks + PF);
                acc[b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rf[ks], rop[b][ks], acc[b], 0, 0, 0);
                if ((k & 3) == 1 && (k >> 2) < NI && !(kLLAblate & 4) && t + 2 < t1) {
                    piece(t + 2, nxt, k >> 2, pa, pb);
                    if (recw && (k >> 2) == 0) records(t + 2, nxt);
                }
                if (DP && k == NGS - 4) tf[0] = hs_tr(old, trb0, trb1, u0);
                if (DP && k == NGS - 2 && CB > 1) tf[1] = hs_tr(old, trb0, trb1, u0 + 1);
            } else if (k < NG) {
                const int cb = k - NGS;
                if (!DS && cb == 0) {
                    tf[0] = hs_tr(old, trb0, trb1, u0);
                    if (CB > 1) tf[1] = hs_tr(old, trb0, trb1, u0 + 1);
                }
                if (cb + 2 < CB) tf[cb + 2] = hs_tr(old, trb0, trb1, u0 + cb + 2);
                acc2[cb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(tf[cb], xsf, acc2[cb], 0, 0, 0);
                if (DS && (cb == 1 || cb == 2))  // S(t)'s partials: [group][writer][block]
                    reinterpret_cast<f32x4_t*>(xw + ((grp * 4 + q) * 2 + cb - 1) * 1024)[lane] = acc[cb - 1];
            }
            if (DX) {
                constexpr int XK0 = DP ? NGS + 1 : (NGS >= NXM ? NGS - NXM : 0);
#pragma unroll
                for (int m = 0; m < NXM; ++m)
                    if (k == XK0 + m) xmicro(m);
            }
            __builtin_amdgcn_sched_barrier(0);
#if LL_STAMP
            if (FL == 7 && k == NGS - 1) {
                unsigned long long tsx = 0;
                LL_TS(tsx);
                hst[1] += tsx - hts1;
                hts1 = tsx;
            }
#endif
        }
        if (DS && (!DP || CB < 3)) {  // no P MFMAs (or too few) to carry them: S(t)'s partials now
#pragma unroll
            for (int b = (DP ? CB - 1 : 0); b < 2; ++b)
                reinterpret_cast<f32x4_t*>(xw + ((grp * 4 + q) * 2 + b) * 1024)[lane] = acc[b];
        }
        if (DX) {  // micro-steps the gaps did not hold
            constexpr int XK0 = DP ? NGS + 1 : (NGS >= NXM ? NGS - NXM : 0);
#pragma unroll
            for (int m = 0; m < NXM; ++m)
                if (XK0 + m >= NG) xmicro(m);
        }
#if LL_STAMP
        if (FL == 7) {
            unsigned long long tsx = 0;
            LL_TS(tsx);
            hst[2] += tsx - hts1;
            hst[3] += 1;
        }
#endif
    };
    auto phase = [&](auto fl_tag, int t) __attribute__((always_inline)) {
#if LL_STAMP
        LL_TS(hts0);
#endif
        // tile t landed (this wave's pieces; the barrier: everyone's); the younger tile's pieces
        // (issued by the previous phase) stay in flight
        // (past the split no tile is fetched at all: a load whose every lane is out of range is
        // not counted in order with the others — measured: the counted wait then let a real
        // tile's reads run ahead of its data)
        if (decltype(fl_tag)::value == 4 || t + 1 >= t1)
            __builtin_amdgcn_s_waitcnt(ll_vmcnt(0));
        else if (recw)
            __builtin_amdgcn_s_waitcnt(ll_vmcnt(NI + 1));
        else
            __builtin_amdgcn_s_waitcnt(ll_vmcnt(NI));
        ll_lds_barrier();
#if LL_STAMP
        LL_TS(hts1);
        if (decltype(fl_tag)::value == 7) hst[0] += hts1 - hts0;
#endif
        body(fl_tag, t, slot_of(t), slot_of(t - 2), slot_of(t - 1), slot_of(t + 2), xbuf + (t & 1) * G::kXBuf,
             xbuf + ((t - 1) & 1) * G::kXBuf, xsb + ((t - 1) & 1) * G::kXs, xsb + ((t - 2) & 1) * G::kXs);
    };
    if (t0 >= t1) return;
    // the register operand has landed before the first tile's DMA: the phase waits count DMA ops
    // only (a load the compiler sank below the prologue's pieces would be the youngest op)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(rop[b][ks]));
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {  // prologue: tiles t0 and t0+1
        if (t0 + tt >= t1) break;
        char* s0 = slot_of(t0 + tt);
        const int m = (t0 + tt) * 16 + rA;
        const int ra0 = ROLE == kHsDw ? tok_row(m) : 0, rb0 = ROLE == kHsDw ? tok_row(m + 8) : 0;
#pragma unroll
        for (int k = 0; k < NI; ++k) piece(t0 + tt, s0, k, ra0, rb0);
        if (recw) records(t0 + tt, s0);
    }
    if (ROLE == kHsDw && a.rows) {  // tile t0+2's row indices
        nrowA = a.rows[min((t0 + 2) * 16 + rA, nv - 1)];
        nrowB = a.rows[min((t0 + 2) * 16 + 8 + rA, nv - 1)];
    }
    using F1 = std::integral_constant<int, 1>;
    using F3 = std::integral_constant<int, 3>;
    using F7 = std::integral_constant<int, 7>;
    using F6 = std::integral_constant<int, 6>;
    using F2 = std::integral_constant<int, 2>;
    using F4 = std::integral_constant<int, 4>;
    phase(F1{}, t0);
    if (t0 + 1 < t1) {
        phase(F3{}, t0 + 1);
        for (int t = t0 + 2; t < t1; ++t) phase(F7{}, t);
        phase(F6{}, t1);
    } else {
        phase(F2{}, t1);
    }
    phase(F4{}, t1 + 1);
#if LL_STAMP
    {
        const int slot = int(blockIdx.x) * 8 + w;
        if (lane == 0 && slot < (1 << 12))
            for (int k = 0; k < 4; ++k) g_ll_stamps[(ROLE == kHsDw ? (1 << 15) : 0) + slot * 8 + k] = hst[k];
    }
#endif
}

template <class G>
__global__ __launch_bounds__(512, 2) void k_lmloss_dw_hs8(LmLossArgs a) {
    constexpr int KS = G::KS, CB = G::CB, HS = G::HS;
    __shared__ __attribute__((aligned(16))) char smem[G::kLds];
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = w >> 2, q = w & 3;
    const int g = lane >> 4, c = lane & 15;
    const int nv = a.rows ? *a.nrows : a.N;
    const bool part = int(blockIdx.x) >= a.dw_full;
    const int j = int(blockIdx.x) - a.dw_full;
    const int vb = part ? a.dw_full + j / a.tsplit : int(blockIdx.x);
    const int ts = part ? j % a.tsplit : 0, nts = part ? a.tsplit : 1;
    const int v0 = vb * 64;
    const int ntt = (nv + 15) / 16;
    const int t0 = int(int64_t(ts) * ntt / nts), t1 = int(int64_t(ts + 1) * ntt / nts);
    bf16x8_t wf[2][KS];  // B operand of S: W[v0 + 32grp + 16b + c][q·HS + 32ks + 8g .. +7]
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int v = v0 + 32 * grp + 16 * b + c;
        const uint16_t* wp = a.w + int64_t(v < a.V ? v : 0) * a.ldw + q * HS + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
            wf[b][ks] = v < a.V ? *reinterpret_cast<const bf16x8_t*>(wp + 32 * ks) : bf16x8_t{};
    }
    f32x16_t acc2[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc2[cb] = f32x16_t{};
    HsFwdState fs{};
    hs8_engine<G, kHsDw, false>(a, smem, wf, acc2, t0, t1, w, v0, nv, fs);
    const int hi = lane >> 5;
    const int vr = 32 * grp + (lane & 31), v = v0 + vr;
#pragma unroll
    for (int cb = 0; cb < CB; ++cb)
#pragma unroll
        for (int r4 = 0; r4 < 4; ++r4) {
            const int col = q * HS + 32 * cb + 8 * r4 + 4 * hi;
            const f32x4_t d = {acc2[cb][4 * r4], acc2[cb][4 * r4 + 1], acc2[cb][4 * r4 + 2], acc2[cb][4 * r4 + 3]};
            if (part) {
                *reinterpret_cast<f32x4_t*>(a.dwpart + (int64_t(j) * 64 + vr) * a.H + col) = d;
            } else if (v < a.V) {
                const int64_t o = int64_t(v) * a.lddw + col;
                if (a.dw_dtype == TRLX_F32)
                    *reinterpret_cast<f32x4_t*>(static_cast<float*>(a.dw) + o) = d;
                else
                    *reinterpret_cast<uint2*>(static_cast<uint16_t*>(a.dw) + o) =
                        make_uint2(pack_bf2(d.x, d.y), pack_bf2(d.z, d.w));
            }
        }
}

template <class G, bool RESTART>
__device__ __forceinline__ void hs8_fwd_block(const LmLossArgs& a, char* smem, int lin, int ntb, int nsplit, int nv) {
    constexpr int KS = G::KS, CB = G::CB, HS = G::HS;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = w >> 2, q = w & 3;
    const int g = lane >> 4, c = lane & 15;
    const int split = lin / ntb, mt = lin - split * ntb;
    const int m0 = mt * kLLTokBlock;
    bf16x8_t hf[2][KS];  // B operand of S: h[token m0 + 32grp + 16b + c][q·HS + 32ks + 8g .. +7]
#pragma unroll
    for (int b = 0; b < 2; ++b) {
        const int tm = m0 + 32 * grp + 16 * b + c, tc = tm < nv ? tm : nv - 1;
        const int row = a.rows ? a.rows[tc] : tc;
        const uint16_t* hp = a.h + int64_t(row) * a.ldh + q * HS + 8 * g;
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) hf[b][ks] = *reinterpret_cast<const bf16x8_t*>(hp + 32 * ks);
    }
    const int nvt = (a.V + 15) / 16;
    const int t0 = int(int64_t(split) * nvt / nsplit), t1 = int(int64_t(split + 1) * nvt / nsplit);
    // the token whose softmax state this lane carries (owner view: 8q + (lane&7) of the group)
    const int town = m0 + 32 * grp + 8 * q + (lane & 7);
    const bool vown = town < nv;
    HsFwdState fs;
    fs.mfix = -INFINITY;
    fs.mtrue = -INFINITY;
    fs.lrun = 0.0f;
    fs.bad = false;
    if (RESTART) fs.mfix = a.mlpart[int64_t(split) * a.N + (vown ? town : nv - 1)].x;
    f32x16_t acc2[CB];
#pragma unroll
    for (int cb = 0; cb < CB; ++cb) acc2[cb] = f32x16_t{};
    hs8_engine<G, kHsFwd, RESTART>(a, smem, hf, acc2, t0, t1, w, 0, nv, fs);
    bool any = false;
    if (!RESTART) {
        any = __any(fs.bad);
        if (lane == 0) a.flags[lin * 8 + w] = any;
    }
    const float mrun = any ? fs.mtrue : fs.mfix;
    // the token's Σ over its 8 lanes (l ^ 8, l ^ 16, l ^ 32)
    float lt = fs.lrun + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, fs.lrun),
                                                                                0x128, 0xf, 0xf, false));
    {
        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(lt), __float_as_uint(lt), false, false);
        lt = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    }
    lt = ll_pair_sum(lt);
    if (vown && lane < 8) a.mlpart[int64_t(split) * a.N + town] = make_float2(mrun, lt);
    const int hi = lane >> 5;
    const int tm = m0 + 32 * grp + (lane & 31);
    if (tm < nv) {
        float* op = a.opart + (int64_t(split) * a.N + tm) * a.H + q * HS + 4 * hi;
#pragma unroll
        for (int cb = 0; cb < CB; ++cb)
#pragma unroll
            for (int r4 = 0; r4 < 4; ++r4)
                *reinterpret_cast<f32x4_t*>(op + 32 * cb + 8 * r4) =
                    f32x4_t{acc2[cb][4 * r4], acc2[cb][4 * r4 + 1], acc2[cb][4 * r4 + 2], acc2[cb][4 * r4 + 3]};
    }
}

template <class G, bool RESTART>
__global__ __launch_bounds__(512, 2) void k_lmloss_fwd_hs8(LmLossArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[G::kLds];
    const int nv = a.rows ? *a.nrows : a.N;
    const int ntb = (nv + kLLTokBlock - 1) / kLLTokBlock;
    const int nsplit = ll_fwd_splits(a, ntb);
    const int total = ntb * nsplit;
    if (!RESTART) {
        const int per_xcd = (total + 7) / 8;
        const int kx = int(blockIdx.x) >> 3, lin = (int(blockIdx.x) & 7) * per_xcd + kx;
        if (kx >= per_xcd || lin >= total) return;
        hs8_fwd_block<G, false>(a, smem, lin, ntb, nsplit, nv);
        return;
    }
    for (int lin = int(blockIdx.x); lin < total; lin += int(gridDim.x)) {
        int f = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) f |= a.flags[lin * 8 + w];
        if (!f) continue;
        hs8_fwd_block<G, true>(a, smem, lin, ntb, nsplit, nv);
        ll_lds_barrier();
    }
}

// ------------------------------------------------------------------ host side
static TuneKnob g_ll_splits{0};  // tuning "lmloss_splits" (0 = auto)
static TuneKnob g_ll_tsplit{0};  // tuning "lmloss_dw_tsplit" (0 = auto)
// tuning "lmloss_fwd": 0 auto (= 2), 1 the 32x32x16 pair form (ll_fwd_block), 2 the 16x16x32 form
// (ll_fwd16_block: no exchange; since the conflict-free image of round 4 the faster one —
// interleaved A/B C2 917-921 vs 938-941 us, C3 625 vs 642 us, profiles/r05b_forms_*), 3 the
// H-sliced form (k_lmloss_fwd_hs), 4 its 8-wave variant (k_lmloss_fwd_hs8).  The saved-P plan
// always runs form 2 (the P layout is that form's).
static TuneKnob g_ll_fwd{0};
// tuning "lmloss_dw": 0 auto (= 4 where the caller's workspace holds the saved P — the PPO
// entries given trlx_ppo_loss_from_hidden_workspace_bytes — else 1), 1 the row-split 16x16x32
// form (k_lmloss_dw: Sᵀ recomputed), 2 / 3 the H-sliced forms (k_lmloss_dw_hs / _hs8), 4 the
// saved-P plan (k_lmloss_dwp; falls back to 1 when the workspace is too small)
static TuneKnob g_ll_dw{0};
// tuning "lmloss_dwp_rw": the saved-P dW kernel's vocab rows per wave, 16·RW (0 auto = 2, 1, 2)
static TuneKnob g_ll_rw{0};

int lmloss_set_tuning(const char* key, int64_t value, bool* handled) {
    const bool sp = key && !__builtin_strcmp(key, "lmloss_splits");
    const bool ts = key && !__builtin_strcmp(key, "lmloss_dw_tsplit");
    const bool fw = key && !__builtin_strcmp(key, "lmloss_fwd");
    const bool dwk = key && !__builtin_strcmp(key, "lmloss_dw");
    const bool rwk = key && !__builtin_strcmp(key, "lmloss_dwp_rw");
    *handled = sp || ts || fw || dwk || rwk;
    if (rwk) {
        TRLX_REQUIRE(value >= 0 && value <= 2, TRLX_ERR_ARG, "lmloss_dwp_rw: 0 auto, 1, 2");
        g_ll_rw = int(value);
        return TRLX_OK;
    }
    if (fw) {
        TRLX_REQUIRE(value >= 0 && value <= 4, TRLX_ERR_ARG,
                     "lmloss_fwd: 0 auto, 1 32x32 pair form, 2 16x16 form, 3 H-sliced form, 4 H-sliced 8-wave form");
        g_ll_fwd = int(value);
        return TRLX_OK;
    }
    if (dwk) {
        TRLX_REQUIRE(value >= 0 && value <= 4, TRLX_ERR_ARG,
                     "lmloss_dw: 0 auto, 1 row-split form, 2 H-sliced form, 3 H-sliced 8-wave form, 4 saved P");
        g_ll_dw = int(value);
        return TRLX_OK;
    }
    if (sp) {
        TRLX_REQUIRE(value >= 0 && value <= kLLMaxSplits, TRLX_ERR_ARG, "lmloss_splits: 0..%d", kLLMaxSplits);
        g_ll_splits = int(value);
    } else if (ts) {
        TRLX_REQUIRE(value >= 0 && value <= 16, TRLX_ERR_ARG, "lmloss_dw_tsplit: 0..16");
        g_ll_tsplit = int(value);
    }
    return TRLX_OK;
}

static size_t ll_align(size_t x) { return (x + 255) & ~size_t(255); }

struct LlWs {
    float* opart;
    float2* mlpart;
    float* trec;
    int* order;
    int* cnt;
    int* flags;
    float* dwpart;
    uint16_t* pbuf;  // saved-P plan only
    f32x4_t* prec;
};
// Compute units of the current device (the grid plans below).
static int ll_ncu() {
    static thread_local int dev = -1, ncu = 0;
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) return 256;
    if (d != dev) {
        int n = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess || n <= 0) n = 256;
        dev = d;
        ncu = n;
    }
    return ncu;
}

// dW grid plan: whole rounds of workgroups own a vocab block each; the blocks of the last,
// partial round are split over the tokens so that round is (nearly) full instead of a tail of
// a few long workgroups (C2: 786 blocks on 256 CUs = 3 rounds + 18 blocks, the 18 split 14 ways).
struct LlDwPlan {
    int full, tsplit, nblk;  // workgroups = full + nblk·tsplit
};
// parts: workgroups per vocab block (the saved-P RW = 2 form's two hidden halves)
static LlDwPlan ll_dw_plan(int64_t V, int vpw = kLLTokBlock, int parts = 1) {
    const int ncu = std::max(1, ll_ncu() / parts);
    const int nvb = int((V + vpw - 1) / vpw);
    const int rem = nvb % ncu;
    LlDwPlan p{nvb, 1, 0};
    if (g_ll_tsplit == 1 || rem == 0) return p;
    const int ts = g_ll_tsplit ? g_ll_tsplit : std::min(16, ncu / rem);
    if (ts <= 1) return p;
    p.full = nvb - rem;
    p.tsplit = ts;
    p.nblk = rem;
    return p;
}

// 32-token tiles of the saved-P layout: the forward's 64-token blocks, whole
static int ll_pntt(int64_t N) { return int(2 * ((N + kLLTokBlock - 1) / kLLTokBlock)); }

// Workspace carve-up for N tokens (dwpart: the split blocks' fp32 partials).
// fwd = false: the backward's carve-up (trlx_lmhead_logprobs_bwd), no forward partials.
// savep: + the saved-P plan's P tiles (⌈V/64⌉ x 2⌈N/64⌉ x 4 KB: 0.62 GB at C2) and records.
static size_t ll_carve(void* base, int64_t N, int64_t H, int64_t V, LlWs* w, bool fwd = true, bool savep = false) {
    char* p = static_cast<char*>(base);
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char* q = p ? p + off : nullptr;
        off += ll_align(bytes);
        return q;
    };
    LlWs t;
    t.opart = reinterpret_cast<float*>(take(fwd ? size_t(kLLMaxSplits) * N * H * 4 : 0));
    t.mlpart = reinterpret_cast<float2*>(take(fwd ? size_t(kLLMaxSplits) * N * 8 : 0));
    t.trec = reinterpret_cast<float*>(take(size_t(N) * 16));
    t.order = reinterpret_cast<int*>(take(size_t(N + 4) * 4));
    t.cnt = reinterpret_cast<int*>(take(size_t(order_chunks(N) + 1) * 4));
    t.flags = reinterpret_cast<int*>(take(size_t((N + kLLRows - 1) / kLLRows) * kLLMaxSplits * 8 * 4));  // <= 8 waves per workgroup
    const LlDwPlan dp = ll_dw_plan(V), dp2 = ll_dw_plan(V, 2 * kLLTokBlock, 2);  // 64- / 128-row blocks
    t.dwpart = reinterpret_cast<float*>(take(std::max(size_t(dp.nblk) * dp.tsplit * kLLTokBlock,
                                                      size_t(dp2.nblk) * dp2.tsplit * 2 * kLLTokBlock) * H * 4));
    t.pbuf = reinterpret_cast<uint16_t*>(take(savep ? size_t((V + 63) / 64) * ll_pntt(N) * 4096 : 0));
    t.prec = reinterpret_cast<f32x4_t*>(take(savep ? size_t(kLLMaxSplits) * N * 16 : 0));
    if (w) *w = t;
    return off;
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
    // the tile DMAs address hidden / weight rows through 32-bit buffer resources with int byte
    // offsets (and an out-of-range sentinel at 0x7ffff000): both spans must stay below it
    TRLX_REQUIRE(N * ldh * 2 < kLLMaxSpan && V * ldw * 2 < kLLMaxSpan, TRLX_ERR_SHAPE,
                 "fused lm_head loss: hidden (%lld x %lld) or weight (%lld x %lld) rows span >= 2 GB "
                 "(split the tokens into chunks)", (long long)N, (long long)ldh, (long long)V, (long long)ldw);
    return TRLX_OK;
}

// The forward's grid covers the largest split plan (every token live, a.nsplit splits),
// rounded up to whole XCD shares; each workgroup finds its (token block, split) on the device.
template <class G, class HG, class H8>
static int ll_launch_fwd(const LmLossArgs& a, hipStream_t s) {
    const int64_t ntb = (a.N + kLLTokBlock - 1) / kLLTokBlock;
    const unsigned grid = unsigned((ntb * a.nsplit + 7) / 8 * 8);
    if (g_ll_fwd == 4 && !a.pbuf) {
        hipLaunchKernelGGL((k_lmloss_fwd_hs8<H8, false>), dim3(grid), dim3(512), 0, s, a);
        const int rc = check_launch("k_lmloss_fwd_hs8");
        if (rc) return rc;
        hipLaunchKernelGGL((k_lmloss_fwd_hs8<H8, true>), dim3(unsigned(std::min<int64_t>(grid, a.ncu))), dim3(512), 0,
                           s, a);
        return check_launch("k_lmloss_fwd_hs8 restart");
    }
    if (g_ll_fwd == 3 && !a.pbuf) {
        hipLaunchKernelGGL((k_lmloss_fwd_hs<HG, false>), dim3(grid), dim3(256), 0, s, a);
        const int rc = check_launch("k_lmloss_fwd_hs");
        if (rc) return rc;
        hipLaunchKernelGGL((k_lmloss_fwd_hs<HG, true>), dim3(unsigned(std::min<int64_t>(grid, a.ncu))), dim3(256), 0,
                           s, a);
        return check_launch("k_lmloss_fwd_hs restart");
    }
    const bool f16 = g_ll_fwd == 0 || g_ll_fwd == 2;
    void (*first)(LmLossArgs) = a.pbuf ? k_lmloss_fwd<G, false, true, true>
                                : f16  ? k_lmloss_fwd<G, false, true>
                                       : k_lmloss_fwd<G, false, false>;
    void (*restart)(LmLossArgs) = a.pbuf ? k_lmloss_fwd<G, true, true, true>
                                  : f16  ? k_lmloss_fwd<G, true, true>
                                         : k_lmloss_fwd<G, true, false>;
    hipLaunchKernelGGL(first, dim3(grid), dim3(G::kThreads), 0, s, a);
    const int rc = check_launch("k_lmloss_fwd");
    if (rc) return rc;
    hipLaunchKernelGGL(restart, dim3(unsigned(std::min<int64_t>(grid, a.ncu))), dim3(G::kThreads), 0, s, a);
    return check_launch("k_lmloss_fwd restart");
}
template <class G, class HG, class H8>
static int ll_launch_dw(const LmLossArgs& a, hipStream_t s) {
    const dim3 grid(unsigned(a.dw_full + a.dw_nblk * a.tsplit));
    if (a.pbuf) {
        if (a.dw_vpw == 2 * kLLTokBlock)  // 128 rows x H/2 per workgroup: two per vocab block
            hipLaunchKernelGGL((k_lmloss_dwp<G, 2, 2>), dim3(2 * grid.x), dim3(G::kThreads), 0, s, a);
        else
            hipLaunchKernelGGL((k_lmloss_dwp<G, 1, 1>), grid, dim3(G::kThreads), 0, s, a);
        return check_launch("k_lmloss_dwp");
    }
    if (g_ll_dw == 3) {
        hipLaunchKernelGGL(k_lmloss_dw_hs8<H8>, grid, dim3(512), 0, s, a);
        return check_launch("k_lmloss_dw_hs8");
    }
    if (g_ll_dw == 2) {
        hipLaunchKernelGGL(k_lmloss_dw_hs<HG>, grid, dim3(256), 0, s, a);
        return check_launch("k_lmloss_dw_hs");
    }
    hipLaunchKernelGGL(k_lmloss_dw<G>, grid, dim3(G::kThreads), 0, s, a);
    return check_launch("k_lmloss_dw");
}
static int ll_fwd(const LmLossArgs& a, hipStream_t s) {
    return a.H == 512 ? ll_launch_fwd<LlG512, HsG<512>, Hs8G<512>>(a, s) : ll_launch_fwd<LlG768, HsG<768>, Hs8G<768>>(a, s);
}
static int ll_dw(const LmLossArgs& a, hipStream_t s) {
    return a.H == 512 ? ll_launch_dw<LlG512, HsG<512>, Hs8G<512>>(a, s) : ll_launch_dw<LlG768, HsG<768>, Hs8G<768>>(a, s);
}

// the common part: shapes, workspace, optional compaction from the mask
static int ll_setup(LmLossArgs& a, const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                    int64_t H, int64_t V, const int64_t* labels, int64_t lb, const int64_t* compact_mask,
                    void* lm_ws, void* dweight, int dw_dtype, int64_t lddw, LlWs& w, hipStream_t s,
                    bool fwd = true, bool savep = false) {
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
    a.nsplit = g_ll_splits ? g_ll_splits : kLLMaxSplits;
    a.nsplit_fixed = g_ll_splits != 0;
    a.ncu = ll_ncu();
    a.dw_vpw = savep && g_ll_rw != 1 ? 2 * kLLTokBlock : kLLTokBlock;
    const LlDwPlan dp = ll_dw_plan(V, a.dw_vpw, a.dw_vpw / kLLTokBlock);
    a.dw_full = dp.full;
    a.tsplit = dp.tsplit;
    a.dw_nblk = dp.nblk;
    ll_carve(lm_ws, N, H, V, &w, fwd, savep);
    a.dwpart = w.dwpart;
    a.pbuf = savep ? w.pbuf : nullptr;
    a.pntt = ll_pntt(N);
    a.prec = savep ? w.prec : nullptr;
    a.opart = w.opart;
    a.mlpart = w.mlpart;
    a.trec = w.trec;
    a.flags = w.flags;
    // dW rows are stored in runs of 4 columns (16 B fp32, 8 B bf16)
    TRLX_REQUIRE(!dweight || (lddw % 4 == 0 && (reinterpret_cast<uintptr_t>(dweight) & 15) == 0), TRLX_ERR_STRIDE,
                 "dweight must be 16-B aligned with a row stride that is a multiple of 4 elements");
    a.dw = dweight;
    a.lddw = lddw;
    a.dw_dtype = dw_dtype;
    if (compact_mask) {
        rc = launch_order<false>(compact_mask, 1, N, w.cnt, w.order, s);  // mask != 0 rows first
        if (rc) return rc;
        a.rows = w.order;
        a.nrows = w.order + N;
    }
    return TRLX_OK;
}

static int ll_dw_finish(const LmLossArgs& a, void* dweight, int dw_dtype, int64_t lddw, const LlWs& w,
                        hipStream_t s) {
    int rc = ll_dw(a, s);
    if (rc || a.dw_nblk == 0) return rc;
    hipLaunchKernelGGL(k_lmloss_dw_reduce, dim3(1024), dim3(256), 0, s, w.dwpart, a.tsplit, a.dw_nblk, a.dw_full,
                       a.dw_vpw, dweight, dw_dtype, a.V, a.H, lddw);
    return check_launch("k_lmloss_dw_reduce");
}

}  // namespace trlx

using namespace trlx;

extern "C" int64_t trlx_lmhead_loss_workspace_bytes(int64_t N, int64_t H, int64_t V) {
    return int64_t(ll_carve(nullptr, N, H, V, nullptr));
}

extern "C" int64_t trlx_lmhead_loss_bwd_workspace_bytes(int64_t N, int64_t H, int64_t V) {
    return int64_t(ll_carve(nullptr, N, H, V, nullptr, false));
}

extern "C" int64_t trlx_ppo_loss_from_hidden_workspace_bytes(int64_t N, int64_t H, int64_t V) {
    return int64_t(ll_carve(nullptr, N, H, V, nullptr, true, true));
}

// The saved-P plan runs when the tuning allows it and the caller's workspace holds the P tiles.
static bool ll_savep_plan(int64_t N, int64_t H, int64_t V, int64_t lm_bytes) {
    return (g_ll_dw == 0 || g_ll_dw == 4) && lm_bytes >= int64_t(ll_carve(nullptr, N, H, V, nullptr, true, true));
}

extern "C" int trlx_ppo_loss_from_hidden_plan(int64_t N, int64_t H, int64_t V, int64_t lm_workspace_bytes) {
    return ll_savep_plan(N, H, V, lm_workspace_bytes) ? 1 : 0;
}

// The PPO loss side from hidden states, once `a` holds the per-token PPO fields (whitening by
// the unsplit record or the split-beta coefficients): shapes, compaction, the three MFMA
// launches and the combine.
static int ll_ppo_loss(LmLossArgs& a, const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t B,
                       int64_t T, int64_t H, int64_t V, const int64_t* labels, const int64_t* mask,
                       const void* values, int v_dtype, const void* old_values, int ov_dtype, const void* returns,
                       int r_dtype, float cliprange, float cliprange_value, float vf_coef, float* lp_out,
                       void* dhidden, int64_t lddh, int dh_dtype, void* dweight, int dw_dtype, int64_t lddw,
                       float* dvalues, void* workspace, void* lm_workspace, int64_t lm_bytes, hipStream_t s) {
    LlWs w;
    const int64_t N = B * T;
    TRLX_REQUIRE(B > 0 && T > 0, TRLX_ERR_SHAPE, "empty rollout batch");
    TRLX_REQUIRE(a.old_lp && values && old_values && returns && lp_out && dhidden && dweight && dvalues && workspace,
                 TRLX_ERR_ARG, "NULL argument to trlx_ppo_loss_from_hidden");
    TRLX_REQUIRE(dh_dtype == TRLX_BF16 || dh_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dhidden dtype");
    TRLX_REQUIRE(dw_dtype == TRLX_BF16 || dw_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dweight dtype");
    TRLX_REQUIRE(r_dtype == TRLX_F32 || r_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "returns dtype %d", r_dtype);
    TRLX_REQUIRE(lddh % 4 == 0 && lddh >= H && lddw >= H, TRLX_ERR_STRIDE, "gradient row strides");
    // the PPO normaliser is Σ mask (ppo_models.py:162,177), read from the record: without it
    // only the all-ones mask (N) is known here
    TRLX_REQUIRE(a.msum || !mask, TRLX_ERR_ARG,
                 "trlx_ppo_loss_from_hidden: a mask needs the GAE record (its Σ mask normalises the loss)");
    // the plan the caller's workspace holds: the saved-P plan (trlx_ppo_loss_from_hidden_workspace_bytes)
    // unless tuned off, else the recompute plan (trlx_lmhead_loss_workspace_bytes)
    TRLX_REQUIRE(lm_bytes >= int64_t(ll_carve(nullptr, N, H, V, nullptr)), TRLX_ERR_ARG,
                 "lm_workspace of %lld bytes: below trlx_lmhead_loss_workspace_bytes(%lld, %lld, %lld)",
                 (long long)lm_bytes, (long long)N, (long long)H, (long long)V);
    const bool savep = ll_savep_plan(N, H, V, lm_bytes);
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, 1, mask, lm_workspace, dweight, dw_dtype, lddw, w,
                      s, true, savep);
    if (rc) return rc;
    Workspace ws;
    carve_ppo_workspace(workspace, B, T, &ws);
    a.mode = kLLPpo;
    a.mask = mask;
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
    hipLaunchKernelGGL(k_lmloss_combine<kLLPpo>, dim3(unsigned(N)), dim3(unsigned(H / 4)), 0, s, a);
    rc = check_launch("k_lmloss_combine");
    if (rc) return rc;
    return ll_dw_finish(a, dweight, dw_dtype, lddw, w, s);
}

extern "C" int trlx_ppo_loss_from_hidden(
    const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t B, int64_t T, int64_t H, int64_t V,
    const int64_t* labels, const void* old_lp, int old_dtype, const float* adv_raw, const double* stats, int unbiased,
    const int64_t* mask, const void* values, int v_dtype, const void* old_values, int ov_dtype, const void* returns,
    int r_dtype, float cliprange, float cliprange_value, float vf_coef, float* lp_out, void* dhidden, int64_t lddh,
    int dh_dtype, void* dweight, int dw_dtype, int64_t lddw, float* dvalues, void* workspace, void* lm_workspace,
    int64_t lm_workspace_bytes, void* stream) {
    LmLossArgs a = {};
    TRLX_REQUIRE(adv_raw, TRLX_ERR_ARG, "NULL adv_raw");
    a.old_lp = old_lp;
    a.old_dtype = old_dtype;
    a.adv = adv_raw;
    a.stats = stats;
    a.unbiased = unbiased;
    a.msum = stats ? stats + 3 : nullptr;
    return ll_ppo_loss(a, hidden, ldh, weight, ldw, B, T, H, V, labels, mask, values, v_dtype, old_values, ov_dtype,
                       returns, r_dtype, cliprange, cliprange_value, vf_coef, lp_out, dhidden, lddh, dh_dtype, dweight,
                       dw_dtype, lddw, dvalues, workspace, lm_workspace, lm_workspace_bytes, (hipStream_t)stream);
}

extern "C" int trlx_ppo_loss_from_hidden_split(
    const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t B, int64_t T, int64_t H, int64_t V,
    const int64_t* labels, const void* old_lp, int old_dtype, const float* adv0, const float* adv_kl,
    const float* rew_kl, const float* rew_score, const float* coef, const double* stats8, int unbiased,
    const double* ctl_state, float kl_coef, float* coef_out, const double* msum, const int64_t* mask,
    const void* values, int v_dtype, const void* old_values, int ov_dtype, float* rewards, void* returns, int r_dtype,
    float cliprange, float cliprange_value, float vf_coef, float* lp_out, void* dhidden, int64_t lddh, int dh_dtype,
    void* dweight, int dw_dtype, int64_t lddw, float* dvalues, void* workspace, void* lm_workspace,
    int64_t lm_workspace_bytes, void* stream) {
    LmLossArgs a = {};
    TRLX_REQUIRE(adv0 && adv_kl && rew_kl && rew_score && rewards, TRLX_ERR_ARG,
                 "NULL split-beta buffer to trlx_ppo_loss_from_hidden_split");
    TRLX_REQUIRE((coef != nullptr) != (stats8 != nullptr), TRLX_ERR_ARG,
                 "trlx_ppo_loss_from_hidden_split: pass exactly one of coef (stored coefficients) and stats8 "
                 "(the split record the coefficients are derived from)");
    a.old_lp = old_lp;
    a.old_dtype = old_dtype;
    a.adv = adv0;
    a.adv_kl = adv_kl;
    a.rew_kl = rew_kl;
    a.rew_score = rew_score;
    a.rewards_out = rewards;
    a.coef = coef;
    a.wstats = stats8;
    a.wunbiased = unbiased;
    a.wctl = ctl_state;
    a.wbeta = kl_coef;
    a.coef_out = stats8 ? coef_out : nullptr;
    a.msum = msum;
    return ll_ppo_loss(a, hidden, ldh, weight, ldw, B, T, H, V, labels, mask, values, v_dtype, old_values, ov_dtype,
                       returns, r_dtype, cliprange, cliprange_value, vf_coef, lp_out, dhidden, lddh, dh_dtype, dweight,
                       dw_dtype, lddw, dvalues, workspace, lm_workspace, lm_workspace_bytes, (hipStream_t)stream);
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
    hipLaunchKernelGGL(k_lmloss_combine<kLLFwd>, dim3(unsigned(N)), dim3(unsigned(H / 4)), 0, s, a);
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
    TRLX_REQUIRE(grad && lse && e, TRLX_ERR_ARG, "NULL grad / lse / E");
    TRLX_REQUIRE(dhidden || dweight, TRLX_ERR_ARG, "neither dhidden nor dweight requested");
    TRLX_REQUIRE(grad_dtype == TRLX_F32 || grad_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "grad dtype");
    TRLX_REQUIRE(dh_dtype == TRLX_BF16 || dh_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dhidden dtype");
    TRLX_REQUIRE(dw_dtype == TRLX_BF16 || dw_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dweight dtype");
    TRLX_REQUIRE(lddh % 4 == 0 && lddh >= H && lddw >= H, TRLX_ERR_STRIDE, "gradient row strides");
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, lb, nullptr, lm_workspace, dweight, dw_dtype, lddw,
                      w, s, false);
    if (rc) return rc;
    a.mode = kLLBwd;
    a.gin = grad;
    a.gin_dtype = grad_dtype;
    a.lse_io = const_cast<float*>(lse);
    a.ebuf = const_cast<float*>(e);
    a.dh = dhidden;
    a.lddh = lddh;
    a.dh_dtype = dh_dtype;
    hipLaunchKernelGGL(k_lmloss_combine<kLLBwd>, dim3(unsigned(N)), dim3(unsigned(H / 4)), 0, s, a);
    rc = check_launch("k_lmloss_combine");
    if (rc || !dweight) return rc;  // a frozen (or tied elsewhere) lm_head: no dW pass
    return ll_dw_finish(a, dweight, dw_dtype, lddw, w, s);
}

#if LL_STAMP
extern "C" int trlx_debug_ll_stamps(void* dst, int64_t n) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ll_stamps), size_t(n) * 8) == hipSuccess ? 0 : 1;
}
#endif
