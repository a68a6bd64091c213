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
//   k_lmloss_fwd      per 64-token block x vocab split, the online softmax over the split and
//                     the "expected embedding" O = Σ_v exp(x_tv − m) · W_v next to it
//                     (flash-style: S = W_tile·hᵀ and Oᵀ += W_tileᵀ·P on MFMA, 2 passes):
//                     partial (m, l, O) per (token, vocab split); saved-P plan: every bf16 P
//                     tile also goes to HBM in the dW kernel's operand layout
//   k_lmloss_combine  per token: merge the splits -> lse, lp, E = O / l; g_t from the PPO loss
//                     (ppo_token.h, the loss rows' own per-token arithmetic) or from a caller's
//                     d loss / d lp; dh_t = g_t (W[y_t] − E_t); the per-token loss record; the
//                     saved-P plan's per-(split, token) record {g·e^(m_split − lse), g·(1 − p_y), y}
//   k_lmloss_dwp      (saved-P plan, the default) per 128 vocab rows x half the hidden columns:
//                     dS = (y == v) ? g·(1 − p_y) : −q·P from the stored P, dW += dS·h on MFMA
//                     (1 pass) — 3 passes in all, the unfused path's count (logits GEMM, dh GEMM,
//                     dW GEMM) without its ~4·N·V bytes of logits / dlogits traffic
//   k_lmloss_dw       (recompute plan: a caller without room for the 2·N·V-byte P buffer)
//                     S = h_tile·W_tileᵀ recomputed, dS formed in registers, dW += dSᵀ·h
//                     (2 passes): 4 in all
// Deterministic: no atomics, fixed reduction orders.
//
// MFMA v_mfma_f32_16x16x32_bf16 throughout.  A workgroup is 4 waves (one per SIMD, 512
// registers each): forward, 64 tokens — S split over the wave pairs' hidden halves, O over the
// waves' hidden quarters with the four waves' P exchanged through LDS (ll_fwd16_block); dW, 64
// (recompute) or 128 (saved P) vocab rows, each wave's rows over the whole H or half of it.
// The streamed operand (W tiles forward, h tiles in dW) is staged by LDS-DMA into ONE swizzled
// image read both by rows and transposed (ds_read_b64_tr_b16), conflict-free.
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
    int dw_vpw;      // vocab rows per dW vocab block (64; the saved-P plan: 64·RW of its form)
    int dw_hsp;      // workgroups per dW vocab block (the saved-P form's hidden parts)
    int sgran;       // vocab tiles per split granule (ll_split_t0): the dW vocab block's, >= 4
    float* dwpart;
    // saved-P plan (k_lmloss_dwp): the forward stores its bf16 P tiles in the dW kernel's layout
    // (ll_p_store); the combine overwrites each token's label entry with −(1 − p_y)/e' and writes
    // the token's h row scaled per split, hq = −g·e'·h with e' = e^(m_split − lse), so dW = P·hq
    // with no per-element arithmetic in the dW kernel (ll_scale)
    uint16_t* pbuf;  // NULL = the recompute plan (k_lmloss_dw)
    int pntt;        // 32-token tiles of the P layout (2·⌈N / 64⌉)
    uint16_t* hq;    // [kLLMaxSplits][N][H] bf16, compact token index (the combine with g: kLLPpo / kLLBwd)
    float* erec;     // [kLLMaxSplits][N] e' per (split, compact token): the drop-in forward writes, its
                     // backward reads (the saved region)
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
// at 2048·(r>>3) + 512·(ch>>2) + 64·(r&7) + 16·((ch&3) ^ ll16_swz((r>>2)&3)).  The 16x16x32 row
// reads (16 rows x 4 chunks) and transposed reads (rows r, r+4 of a subtile in one 32-lane group)
// are conflict-free on it (the plain (r>>2)&3 swizzle left them 2-way conflicted — PMC:
// SQ_LDS_BANK_CONFLICT = 48 % of the dW kernel's LDS cycles), and the XOR touches only the low 2
// bits of the chunk: every read of a lane is one of 2 base addresses plus an immediate.
__device__ __forceinline__ int ll16_swz(int R) { return (0x78 >> (2 * R)) & 3; }  // 0 2 3 1
// The tile row that lane `lane` of DMA piece i fills (piece i: segment i >> 3, 8-row group
// (i & 7) >> 1, subtile pair i & 1).
__device__ __forceinline__ int ll_piece_row(int i, int lane) { return 8 * ((i & 7) >> 1) + ((lane >> 2) & 7); }
// One 1-KB LDS-DMA piece of a tile: lane l lands at the piece's byte 16·l, so it fetches the
// logical chunk that the image puts there (this function: its byte offset in the row-major
// source, `row_bytes` = the offset of the lane's row).  Buffer-resource form: hipcc then tracks
// these LDS writes and does not put a vmcnt(0) in front of the next LDS read (the flat
// global_load_lds form made every tile wait for the DMA of the NEXT one before its first read).
__device__ __forceinline__ int ll16_piece_src(int i, int row_bytes, int lane) {
    const int r = ll_piece_row(i, lane);
    const int ch = 4 * (2 * (i & 1) + (lane >> 5)) + ((lane & 3) ^ ll16_swz((r >> 2) & 3));
    return row_bytes + (i >> 3) * 256 + ch * 16;
}
// The buffer resource of 32-row tile t of a [rows][ld] bf16 matrix, limited to its rows below
// `nrows` (0: none): rows past it read as zeros by the range check, so a piece's per-lane offset
// within the tile is loop-invariant and the tile is scalar arithmetic only.  (A helper, not a
// lambda in the kernel body: hipcc's host pass dropped the kernels' launch stubs for a lambda
// returning a resource, and the library then linked with undefined symbols.)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t ll_tile_rsrc(const uint16_t* base, int ld, int t, int nrows) {
    // (the clamp compiles to a VALU v_med3: readfirstlane keeps the resource in scalar registers —
    // a resource in vector registers makes hipcc wrap the load in a waterfall loop)
    const int rows = __builtin_amdgcn_readfirstlane(max(0, min(kLLRows, nrows - t * kLLRows)));
    return make_rsrc(base + int64_t(t) * kLLRows * ld, uint32_t(rows) * uint32_t(ld) * 2u);
}
__device__ __forceinline__ void ll16_piece_at(char* slot, int il, __amdgpu_buffer_rsrc_t rs, int off) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(slot + il * 1024), 16, off, 0, 0,
                                             0);
}
__device__ __forceinline__ void ll16_piece(char* slot, int i, __amdgpu_buffer_rsrc_t rs, int row_bytes, int lane) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(slot + i * 1024), 16,
                                             ll16_piece_src(i, row_bytes, lane), 0, 0, 0);
}

__device__ __forceinline__ bf16x8_t pack8(const float* p) {
    bf16x8_t r;
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] = (__bf16)p[j];
    return r;
}

// s_waitcnt immediate for vmcnt(n) alone (gfx9 encoding: vmcnt[3:0] + [15:14], expcnt 7,
// lgkmcnt 15): the builtin, unlike inline asm, is seen by the compiler's own wait insertion.
constexpr int ll_vmcnt(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70; }

// max / sum over the four 16-lane rows (lanes l, l^16, l^32, l^48: one token's four lane groups
// in the 16x16x32 forms), the same bits in every lane.  v_permlane16/32_swap are VALU: a
// __shfl_xor is a ds_bpermute, an LDS round trip whose lgkmcnt(0) also drains the operand reads
// in flight.
__device__ __forceinline__ float ll_pair_max(float v) {  // over lanes l and l^32
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float ll_pair_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float ll_rows_max(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return ll_pair_max(fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1])));
}
__device__ __forceinline__ float ll_rows_sum(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return ll_pair_sum(__uint_as_float(r[0]) + __uint_as_float(r[1]));
}

// A workgroup barrier ordering LDS only.  __syncthreads() and an LDS-scope release fence both
// wait for vmcnt(0) — the tile DMAs still in flight are LDS writes too — so the barrier is
// spelled out: this wave's LDS accesses done, then s_barrier (the memory clobber keeps the
// compiler from moving loads / stores across it).
__device__ __forceinline__ void ll_lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Workgroup geometry: 4 waves (one per SIMD, 512 registers each) over 64 tokens (forward) / 64
// vocab rows (dW); at H = 768 a wave holds 96 h / W fragment registers and 192 accumulators.
template <int H_>
struct LlGeom {
    static constexpr int H = H_;
    static constexpr int kWaves = 4, kThreads = kWaves * 64;
    static constexpr int kPieces = H / 16, NI = kPieces / kWaves;  // 1-KB DMA pieces per tile / per wave
    static constexpr int kStage = kLLRows * H * 2;
    static_assert(kPieces % kWaves == 0 && H % 256 == 0, "geometry: whole 128-column segments per hidden half");
};
typedef LlGeom<768> LlG768;
typedef LlGeom<512> LlG512;

// ------------------------------------------------------------------ 16x16x32 operand reads
// Per-lane byte offsets in a staged 32-row tile (the subtile image above) for
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
// P is stored non-temporal: 2·N·V bytes written once and read once, by k_lmloss_dwp after the
// combine (C2 update −7 %, profiles/r06n_fwd_pstore_nt_ab.log; nt on the O partials and on dW's
// output measured neutral, r06o_opart_dwout_nt_ab.log)
__device__ __forceinline__ void ll_p_store(const LmLossArgs& a, const s16x8_t& v, int t, int tt, int half,
                                           int lane) {
    const int g = lane >> 4, c = lane & 15;
    char* dst = reinterpret_cast<char*>(a.pbuf) +
                ((int64_t(t >> 1) * a.pntt + tt) * 4 + 2 * (t & 1) + (g >> 1)) * 1024 +
                16 * (16 * (2 * half + (g & 1)) + c);
    __builtin_nontemporal_store(v, reinterpret_cast<s16x8_t*>(dst));
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

// Vocab tiles of split s: [ll_split_t0(s), ll_split_t0(s + 1)), whole granules of `gran` tiles
// (a.sgran: the saved-P dW vocab block, 128 or 256 rows), so a dW workgroup's vocab rows never
// straddle two splits (its four waves share one staged tile of the split's scaled h); the largest
// split is at most gran − 1 tiles over the even share.
__device__ __forceinline__ int ll_split_t0(int s, int nvt, int nsplit, int gran) {  // 32-bit: s·ngr < 2^31
    return min(nvt, gran * int(unsigned(s) * unsigned((nvt + gran - 1) / gran) / unsigned(nsplit)));
}
__device__ __forceinline__ int ll_split_of(int vt, int nvt, int nsplit, int gran) {
    int s = 0;
    for (int k = 1; k < nsplit; ++k) s = ll_split_t0(k, nvt, nsplit, gran) <= vt ? k : s;
    return s;
}
// The scale of split s's P for a token: e' = e^(m_s − lse) (a split with no vocab: 0), clamped to
// 2^-100 from below so the label entry −(1 − p_y)/e' stays finite (terms of a split whose
// e^(m_s − lse) underflows are then weighted by 2^-100 instead of less: below any fp32 gradient)
__device__ __forceinline__ float ll_scale(float ms, float lse) {
    return ms == -INFINITY ? 0.0f : fmaxf(exp2_fast((ms - lse) * kLog2e), 0x1p-100f);
}
// P[vocab row v][compact token m] in the saved-P layout (ll_p_store)
__device__ __forceinline__ uint16_t* ll_p_elem(const LmLossArgs& a, int v, int m) {
    const int vt = v >> 5, rr = v & 31, j32 = m & 31;
    return a.pbuf + (((int64_t(vt >> 1) * a.pntt + (m >> 5)) * 4 + 2 * (vt & 1) + (rr >> 4)) * 1024 +
                     16 * (16 * (j32 >> 3) + (rr & 15)) + 2 * (j32 & 7)) / 2;
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
// the softmax's gaps in the S loop (see kSM0 below): first gap and stride of the exps
#ifndef LL_FWD_SM0
#define LL_FWD_SM0 12
#endif
#ifndef LL_FWD_SMS
#define LL_FWD_SMS 3
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
// MFMAs carried across a barrier (O exchange + S pair split): the last LL_FWD_DEFO W^T fragments of
// O(t) (4 MFMAs each) issue after step t+1's first barrier, the last LL_FWD_DEFS MFMAs of S(t+1)
// after step t's exchange barrier, behind the LDS reads each barrier releases (the W rows of tile
// t+1 / the exchanged P), so the matrix pipe runs while those reads are in flight
#ifndef LL_FWD_DEFO
#define LL_FWD_DEFO 1
#endif
#ifndef LL_FWD_DEFS
#define LL_FWD_DEFS 4
#endif
// O exchange: W^T fragments in flight in the O loop (2 reads each; the first ones read in the S
// loop's last gaps)
#ifndef LL_FWD_PFX
#define LL_FWD_PFX 2
#endif
// the S loop gap that adds the partner's partial of S(t) (read after the step's first barrier)
#ifndef LL_FWD_XRG
#define LL_FWD_XRG 4
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
    // softmax(t) in the S loop's gaps: the token max at kSM0, the offset / overflow flag two gaps
    // later, the exps one every kSMS gaps from kSM0 + 3 (the 8th with the row sum and the bf16 pack
    // at kSMP), P(t) to the exchange slot at kSMP + 1
    // (the macros are for H = 768's 48 gaps; scaled to the S loop's gaps at other H)
    constexpr int kSM0 = LL_FWD_SM0 * NG / 48, kSMS = LL_FWD_SMS * NG / 48 > 0 ? LL_FWD_SMS * NG / 48 : 1;
    constexpr int kSMP = kSM0 + 3 + 7 * kSMS;
    constexpr int kPS = LL_FWD_PSTAGE_GAP * NG / 48 > kSMP + 1 ? LL_FWD_PSTAGE_GAP * NG / 48 : kSMP + 2;
    static_assert(kSMS >= 1 && kSMP + 1 < 2 * KS, "the softmax gaps inside the S loop");
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
    static_assert(!PSL || kPS > kSMP + 1, "the saved-P transpose after the exchange slot's write");
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
    const int t0 = ll_split_t0(split, nvt, nsplit, a.sgran), t1 = ll_split_t0(split + 1, nvt, nsplit, a.sgran);
    // one buffer resource per W tile: its rows [32t, min(V, 32t + 32)), none past the split — rows
    // past V and tiles past the split read as zeros by the range check, and a piece's per-lane
    // offset is loop-invariant: the tile is all scalar arithmetic (no VALU per piece)
    auto issue_piece = [&](int t, char* slot, int k) __attribute__((always_inline)) {
        const int i = wave + G::kWaves * k;
        ll16_piece(slot, i, ll_tile_rsrc(a.w, int(a.ldw), t, t < t1 ? a.V : 0), ll_piece_row(i, lane) * int(a.ldw) * 2,
                   lane);
    };
    auto load_piece = [&](int t, int k) __attribute__((always_inline)) {
        const int i = wave + G::kWaves * k;
        return __builtin_amdgcn_raw_buffer_load_b128(ll_tile_rsrc(a.w, int(a.ldw), t, t < t1 ? a.V : 0),
                                                     ll16_piece_src(i, ll_piece_row(i, lane) * int(a.ldw) * 2, lane), 0, 0);
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
    constexpr int PFX = LL_FWD_PFX;
    constexpr int DEFO = OX && SP ? LL_FWD_DEFO : 0, DEFS = OX && SP ? LL_FWD_DEFS : 0;
    static_assert(DEFO >= 0 && DEFO < OF - PFX && DEFS >= 0 && DEFS <= 8, "carried MFMAs");
    // the exchanged P of the four token blocks (held past the step for the carried O fragments)
    bf16x8_t px[4], tfd[DEFO > 0 ? DEFO : 1];
#pragma unroll
    for (int tb = 0; tb < 4; ++tb) px[tb] = bf16x8_t{};
#pragma unroll
    for (int i = 0; i < (DEFO > 0 ? DEFO : 1); ++i) tfd[i] = bf16x8_t{};
    // the carried O MFMAs (zero operands before the first step)
    auto o_carried = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < DEFO; ++i)
#pragma unroll
            for (int tb = 0; tb < 4; ++tb)
                O[4 * (OF - DEFO + i) + tb] =
                    __builtin_amdgcn_mfma_f32_16x16x32_bf16(tfd[i], px[tb], O[4 * (OF - DEFO + i) + tb], 0, 0, 0);
    };
    // NF: the fragments done here (OF, or OF − DEFO with the rest carried); pre: after the P reads
    auto ox_product = [&](const char* tile, bf16x8_t (&tf)[OF], int gbase, auto&& gap, auto&& pre, auto nf_tag)
                          __attribute__((always_inline)) {
        constexpr int NF = decltype(nf_tag)::value;
#pragma unroll
        for (int tb = 0; tb < 4; ++tb) px[tb] = *reinterpret_cast<const bf16x8_t*>(xrd + 4096 * tb);
        pre();
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int f = 0; f < OF; ++f) {
            if (f + PFX < OF) tf[f + PFX] = ox_frag(tile, f + PFX);
            if (f < NF) {
#pragma unroll
                for (int tb = 0; tb < 4; ++tb)
                    O[4 * f + tb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(tf[f], px[tb], O[4 * f + tb], 0, 0, 0);
            } else {
                tfd[f - NF] = tf[f];
            }
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
        for (int e = 0; e < 8; ++e)  // S(t) for the softmax (SP: + the partner's, at gap LL_FWD_XRG); S(t+1) anew
            x[e] = s[e >> 2][e & 3];
        if constexpr (DEFO > 0) {
            __builtin_amdgcn_sched_barrier(0);
            o_carried();  // O(t-1)'s last fragments, behind the reads of tile t+1
            __builtin_amdgcn_sched_barrier(0);
        }
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
            if (SP && k == LL_FWD_XRG) {
#pragma unroll
                for (int e = 0; e < 8; ++e) x[e] += xr[e >> 2][e & 3];
            }
            if (k < NG - DEFS) s_mfma(nx, af, k);
            if (SAVEP && (!SP || PSL) && k == kPS) {
                if (kLLAblate & 64) {  // diagnostic: no LDS round trip (wrong layout)
                    pt = __builtin_bit_cast(s16x8_t, pb);
                } else {
                    pt = p_stage(pb);  // PSL: after the slot write at gap 12
                }
            }
            if (k == kSM0) {  // the lane's max + token max (no mask inside the loop: the last tile's own path)
                const float lm = fmaxf(fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3])),
                                       fmaxf(fmaxf(x[4], x[5]), fmaxf(x[6], x[7])));
                m4 = ll_rows_max(lm);
            } else if (k == kSM0 + 2) {
                sm_chunk(1, t, std::false_type{});
            } else if (k == kSMP) {
                sm_chunk(9, t, std::false_type{});
                sm_chunk(10, t, std::false_type{});
                pb = pack8(pr);
            } else if (OX && k == kSMP + 1) {
                *reinterpret_cast<bf16x8_t*>(xch) = pb;  // the exchange: read after the S loop's barrier
            }
#pragma unroll
            for (int e = 0; e < 7; ++e)
                if (k == kSM0 + 3 + kSMS * e) sm_chunk(2 + e, t, std::false_type{});
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
            }, [&]() __attribute__((always_inline)) {
#pragma unroll
                for (int k = NG - DEFS; k < NG; ++k) s_mfma(nx, af, k);  // S(t+1)'s last, behind the P reads
            }, std::integral_constant<int, OF - DEFO>{});
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
        if (SAVEP && !(kLLAblate & 32)) ll_p_store(a, pt, t, ptt, phalf, lane);  // after the O loop
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
        o_carried();  // the last step's carried O fragments
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
            ox_product(c0, tfx, 0, [](int) {}, []() {}, std::integral_constant<int, OF>{});
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
template <class G, bool RESTART, bool SAVEP>
__global__ __launch_bounds__(G::kThreads, 1) void k_lmloss_fwd(LmLossArgs a) {
    __shared__ __attribute__((aligned(16))) char smem[3 * G::kStage + G::kWaves * 4096];
    static_assert(3 * G::kStage + G::kWaves * 4096 <= 163840, "forward LDS: 3 stages + exchange");
    const int nv = a.rows ? *a.nrows : a.N;
    const int ntb = (nv + kLLTokBlock - 1) / kLLTokBlock;
    const int nsplit = ll_fwd_splits(a, ntb);
    const int total = ntb * nsplit;
    if (!RESTART) {
        const int per_xcd = (total + 7) / 8;
        const int kx = int(blockIdx.x) >> 3, lin = (int(blockIdx.x) & 7) * per_xcd + kx;
        if (kx >= per_xcd || lin >= total) return;  // past an XCD's share / the live tokens
        ll_fwd16_block<G, false, SAVEP>(a, smem, lin, ntb, nsplit, nv);
        return;
    }
    for (int lin = int(blockIdx.x); lin < total; lin += int(gridDim.x)) {
        int f = 0;
#pragma unroll
        for (int w = 0; w < G::kWaves; ++w) f |= a.flags[lin * G::kWaves + w];
        if (!f) continue;
        ll_fwd16_block<G, true, SAVEP>(a, smem, lin, ntb, nsplit, nv);
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
// 8 waves a SIMD (≤ 64 VGPRs): one more wave of loads in flight than the 65 registers hipcc picks
// by itself allow (−3.5 µs of ~50 at C2, profiles/r06w8_combine_occupancy_kab.log)
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void k_lmloss_combine(LmLossArgs a) {
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
        if (MODE == kLLFwd) {  // the drop-in's skipped token: lp = lse = 0 (its E is never read)
            if (d4 == 0) {
                st_any(a.lp, a.lp_dtype, row, 0.0f);
                if (a.lse_io) a.lse_io[row] = 0.0f;
            }
            return;
        }
        if (!a.dh) return;
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
        // the saved-P plan: the split scales e' and the label entry of P (ll_scale)
        float es[kLLMaxSplits];
#pragma unroll
        for (int s = 0; s < kLLMaxSplits; ++s) es[s] = s < nsplit ? ll_scale(ml[s].x, lse) : 0.0f;
        if (a.pbuf && d4 == 0 && yok) {
            const int nvt = (a.V + kLLRows - 1) / kLLRows, sy = ll_split_of(int(y) >> 5, nvt, nsplit, a.sgran);
            float ey = es[0];
#pragma unroll
            for (int s = 1; s < kLLMaxSplits; ++s) ey = sy == s ? es[s] : ey;
            *ll_p_elem(a, int(y), m) = f2bf(expm1f(lp) / ey);  // −(1 − p_y)/e'
        }
        if (MODE == kLLPpo) {
            PolicyTerms pt;
            g = ppo_policy_dlp(lp, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
            if (a.hq) {  // the token's h scaled per split: hq = −g·e'·h
#pragma unroll
                for (int s = 0; s < kLLMaxSplits; ++s) {
                    if (s >= nsplit) break;
                    const float q = -g * es[s];
                    reinterpret_cast<uint2*>(a.hq + (int64_t(s) * a.N + m) * a.H)[d4] =
                        make_uint2(pack_bf2(q * bf_lo(hv.x), q * bf_hi(hv.x)), pack_bf2(q * bf_lo(hv.y), q * bf_hi(hv.y)));
                }
            }
            if (d4 == 0) {
                const bool masked = p.m == 0.0f;
                a.lp_out[row] = masked ? 0.0f : lp;
                if (masked) ppo_policy_dlp(0.0f, p.olp, p.A, p.m, p.inv_msum, a.cliprange, pt);
                token_record(a, row, pt, p, vin);
                if (a.coef || a.wstats) split_outputs(a, row, p);
            }
        } else {  // kLLFwd
            if (a.erec && d4 < nsplit) {  // the drop-in: e' kept for the backward (which knows g)
                float ed = es[0];
#pragma unroll
                for (int s = 1; s < kLLMaxSplits; ++s) ed = d4 == s ? es[s] : ed;
                a.erec[int64_t(d4) * a.N + m] = ed;
            }
            if (d4 == 0) {
                st_any(a.lp, a.lp_dtype, row, lp);
                if (a.lse_io) a.lse_io[row] = lse;
            }
        }
    } else {  // kLLBwd: lse from the forward, g = the caller's d loss / d lp
        e = reinterpret_cast<const f32x4_t*>(a.ebuf + int64_t(row) * a.H)[d4];
        lse = a.lse_io[row];
        g = ld_any(a.gin, a.gin_dtype, row);
        if (a.hq) {  // the saved-P plan: hq = −g·e'·h from the forward's e'
            nsplit = ll_fwd_splits(a, (nv + kLLTokBlock - 1) / kLLTokBlock);
            const uint2 hv = reinterpret_cast<const uint2*>(a.h + int64_t(row) * a.ldh)[d4];
#pragma unroll
            for (int s = 0; s < kLLMaxSplits; ++s) {
                if (s >= nsplit) break;
                const float q = -g * a.erec[int64_t(s) * a.N + m];
                reinterpret_cast<uint2*>(a.hq + (int64_t(s) * a.N + m) * a.H)[d4] =
                    make_uint2(pack_bf2(q * bf_lo(hv.x), q * bf_hi(hv.x)), pack_bf2(q * bf_lo(hv.y), q * bf_hi(hv.y)));
            }
        }
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
    // per-lane byte offsets in a staged tile (the subtile image above):
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

// A 16-B buffer load: uniform resource and offset, per-lane offset (no 64-bit address register)
__device__ __forceinline__ s16x8_t ll_buf_load16(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
    return __builtin_bit_cast(s16x8_t, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0));
}

// ------------------------------------------------------------------ dW from the saved P
// dW = Σ_t dS_t·h_t with dS = (y == v) ? g·(1 − p_y) : −g·e^(m_split − lse)·P, regrouped so the
// dW kernel does no arithmetic on its operands: the forward left every bf16 P tile in HBM in this
// kernel's A-operand layout (ll_p_store), the combine overwrote each token's label entry with
// −(1 − p_y)/e' and wrote the token's h row scaled per vocab split, hq_s = −g·e'_s·h (e' =
// e^(m_s − lse), ll_scale), so
//   dW[v] = Σ_t P[v][t] · hq_{split(v)}[t]          (label entries: −(1 − p_y)/e' · −g·e'·h = g·(1 − p_y)·h)
// — ONE plain MFMA product per 32-token tile: the A operand is the P chunk as loaded (one 16-B
// load a lane, three tiles ahead), the B operand the staged hq tile read transposed.  Numerics as
// the per-element form it replaced (round 5: dS formed from P and a per-(split, token) record in
// the MFMA gaps, ~430 of its 1,910 cycles a tile): one bf16 rounding on each side of every product
// (P, and hq instead of dS).  Workgroup = 64·RW vocab rows (4 waves x 16·RW rows; HSP = 2: half the
// hidden columns, the two halves adjacent in dispatch order so the second P read hits the
// Infinity Cache) x one token split; its rows lie in one vocab split (ll_split_t0's 128-row
// granules), so the four waves share each staged hq tile.  3-stage hq ring (the DMA of tile t+2
// during tile t) and counted vmcnt: the barrier waits only for what was issued before the
// previous tile.
// transposed hq fragments in flight: 2 reads each, and lgkmcnt counts to 15 only — at 8 (16
// reads + the next fragment's) hipcc could not express the wait for the oldest and drained the
// whole LDS queue (lgkmcnt(0)) at every tile's first MFMA
#ifndef LL_DWP_PFO
#define LL_DWP_PFO 6
#endif
#ifndef LL_DWP_PIECE_GAP
#define LL_DWP_PIECE_GAP 4
#endif
#ifndef LL_DWP_PIECE_OFF
#define LL_DWP_PIECE_OFF 1
#endif
template <class G, int RW, int HSP>
__global__ __launch_bounds__(256, 1) void k_lmloss_dwp(LmLossArgs a) {
    constexpr int H = G::H, HC = H / HSP, DB = HC / 16, NI = G::NI / HSP;
    constexpr int kStage = G::kStage / HSP;
    static_assert(G::kWaves == 4, "dW: four waves per workgroup");
    static_assert(HC % 128 == 0, "h parts of whole 128-column segments");
    static_assert(3 * kStage <= 163840, "3 hq stages");
    // the next-but-one tile's hq pieces every kPG-th gap from kPO on
    constexpr int kPG = LL_DWP_PIECE_GAP, kPO = LL_DWP_PIECE_OFF;
    static_assert(kPO < kPG && kPG * (NI - 1) + kPO < DB, "every DMA piece inside the tile's gaps");
    __shared__ __attribute__((aligned(16))) char smem[3 * kStage];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int g = lane >> 4, c = lane & 15, q = (lane >> 2) & 3, p = lane & 3;
    // the live token count, uniform (readfirstlane tells hipcc so: the tile resources below
    // derive from it, and a resource in vector registers makes it wrap every buffer load in a
    // waterfall loop)
    const int nv = __builtin_amdgcn_readfirstlane(a.rows ? *a.nrows : a.N);
    constexpr int vpw = 64 * RW;
    // the block and hidden part of this workgroup (the parts adjacent in dispatch order)
    const int hp = HSP == 1 ? 0 : int(blockIdx.x) % HSP, bid = int(blockIdx.x) / HSP;
    const bool part = bid >= a.dw_full;
    const int j = bid - a.dw_full;
    const int vb = part ? a.dw_full + j / a.tsplit : bid;
    const int ts = part ? j % a.tsplit : 0, nts = part ? a.tsplit : 1;
    const int r0 = vb * vpw + wave * 16 * RW;  // this wave's first vocab row
    const int ntt = (nv + kLLRows - 1) / kLLRows;
    const int t0 = int(int64_t(ts) * ntt / nts), t1 = int(int64_t(ts + 1) * ntt / nts);
    // the vocab split of the workgroup's rows (the forward's plan, ll_fwd_splits / ll_split_t0)
    // (ll_fwd_splits' float arithmetic runs on the VALU: readfirstlane keeps the split uniform)
    const int nsplit = __builtin_amdgcn_readfirstlane(ll_fwd_splits(a, (nv + kLLTokBlock - 1) / kLLTokBlock));
    const int sp = __builtin_amdgcn_readfirstlane(ll_split_of((vb * vpw) >> 5, (a.V + kLLRows - 1) / kLLRows, nsplit, a.sgran));
    // transposed reads of the hq tile: rows 8g + 4hf + q, columns 16nb + 4p (the subtile image)
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
    // one buffer resource per hq tile: this split's rows of the tile's live tokens [32t, min(nv,
    // 32t + 32)), none past the token split — the rest read as zeros by the range check, and a
    // piece's per-lane offset is loop-invariant: the tile is all scalar arithmetic (ll_hq_fits
    // keeps the whole hq buffer below the 2 GB sentinel)
    const uint16_t* hq0 = a.hq + int64_t(sp) * a.N * H;
    auto stage = [&](int t) __attribute__((always_inline)) { return smem + (t % 3) * kStage; };
    // piece il of the part's image = piece hp·HC/16 + il of the full-H image (a multiple of 8:
    // the same rows).  Issued unconditionally — a branch around it would leave hipcc unable to
    // count the loads in flight across the loop and it would wait for all of them (vmcnt(0))
    // instead of the counted waits
    auto issue_piece = [&](int t, char* slot, int k) __attribute__((always_inline)) {
        const int il = wave + G::kWaves * k;
        ll16_piece_at(slot, il, ll_tile_rsrc(hq0, H, t, t < t1 ? nv : 0),
                      ll16_piece_src(hp * (HC / 16) + il, ll_piece_row(il, lane) * (H * 2), lane));
    };
    // P chunk of tile t for row half hh (rows r0 + 16hh + c, tokens 8g..8g+7), clamped to the
    // split's last tile: 64-row block (r0 + 16hh) / 64, dW wave slot ((r0 + 16hh) / 16) & 3.  A
    // uniform base plus the lane's 16 B: no per-tile address register (a temporary that reused a
    // P destination made hipcc wait for the previous tile's P loads every fourth tile)
    const __amdgpu_buffer_rsrc_t rp =
        make_rsrc(reinterpret_cast<const char*>(a.pbuf) + (int64_t(r0 >> 6) * a.pntt * 4 + ((r0 >> 4) & 3)) * 1024,
                  uint32_t(a.pntt) * 4096u);  // this block's token tiles (128·N B)
    const int plane = 16 * lane;
    auto load_p = [&](int t, int hh) __attribute__((always_inline)) {
        return ll_buf_load16(rp, plane, min(t, t1 - 1) * 4096 + 1024 * hh);
    };
    f32x4_t D[RW][DB];  // dW[r0 + 16hh + 4g + r][16nb + c]
#pragma unroll
    for (int hh = 0; hh < RW; ++hh)
#pragma unroll
        for (int nb = 0; nb < DB; ++nb) D[hh][nb] = f32x4_t{};
    s16x8_t R0[RW], R1[RW], R2[RW], R3[RW];  // P(t0 + k) in R[k % 4]
#pragma unroll
    for (int hh = 0; hh < RW; ++hh) R0[hh] = R1[hh] = R2[hh] = R3[hh] = s16x8_t{};
    if (t0 < t1) {
#pragma unroll
        for (int hh = 0; hh < RW; ++hh) {
            R0[hh] = load_p(t0, hh);
            R1[hh] = load_p(t0 + 1, hh);
            R2[hh] = load_p(t0 + 2, hh);
        }
#pragma unroll
        for (int k = 0; k < NI; ++k) issue_piece(t0, stage(t0), k);
#pragma unroll
        for (int k = 0; k < NI; ++k) issue_piece(t0 + 1, stage(t0 + 1), k);
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(0));
        ll_lds_barrier();
    }
    // tile t: dW += P(t)·hq(t) with P(t) in `use`; in its gaps the DMA of tile t+2 (fut) and the
    // P loads of tile t+3 (into `nw`).  The LDS regions are __restrict__ parameters (alias scopes:
    // hipcc otherwise waits for the DMA before every read of the current tile).
    auto tile_body = [&](const char* __restrict__ cur, char* __restrict__ fut, int t, const s16x8_t (&use)[RW],
                         s16x8_t (&nw)[RW]) __attribute__((always_inline)) {
        constexpr int PFO = LL_DWP_PFO;
        bf16x8_t da[RW], tf[DB];
#pragma unroll
        for (int hh = 0; hh < RW; ++hh) da[hh] = __builtin_bit_cast(bf16x8_t, use[hh]);
#pragma unroll
        for (int nb = 0; nb < PFO; ++nb) tf[nb] = tr_frag(cur, nb);
#pragma unroll
        for (int nb = 0; nb < DB; ++nb) {
            if (nb + PFO < DB) tf[nb + PFO] = tr_frag(cur, nb + PFO);
#pragma unroll
            for (int hh = 0; hh < RW; ++hh)
                D[hh][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[hh], tf[nb], D[hh][nb], 0, 0, 0);
            if (nb == 0) {
#pragma unroll
                for (int hh = 0; hh < RW; ++hh) nw[hh] = load_p(t + 3, hh);
            }
            if (nb % kPG == kPO && nb / kPG < NI) issue_piece(t + 2, fut, nb / kPG);
            __builtin_amdgcn_sched_barrier(0);
        }
    };
    auto tile = [&](int t, const s16x8_t (&use)[RW], s16x8_t (&nw)[RW]) __attribute__((always_inline)) {
        // everything issued before the previous tile's body (RW P loads + NI pieces a tile):
        // hq(t) and P(t)
        __builtin_amdgcn_s_waitcnt(ll_vmcnt(NI + RW));
        ll_lds_barrier();
        tile_body(stage(t), stage(t + 2), t, use, nw);
    };
    // (tiles 2-4 of a group conditional: unconditional groups padded with empty tiles, or a
    // 1-3 tile tail after the loop, spared hipcc's wait analysis a conservative vmcnt at each
    // group's first MFMA but made it rotate the dW accumulators between registers every tile —
    // ~40 moves a tile, 3-4 % slower: profiles/r06e_dwp_loop_ab.log)
    for (int t = t0; t < t1; t += 4) {
        tile(t, R0, R3);
        if (t + 1 < t1) tile(t + 1, R1, R0);
        if (t + 2 < t1) tile(t + 2, R2, R1);
        if (t + 3 < t1) tile(t + 3, R3, R2);
    }
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

// ------------------------------------------------------------------ host side
static TuneKnob g_ll_splits{0};  // tuning "lmloss_splits" (0 = auto)
static TuneKnob g_ll_tsplit{0};  // tuning "lmloss_dw_tsplit" (0 = auto)
// tuning "lmloss_dw": 0 auto (= 4 where the caller's buffers hold the saved P — the PPO entries
// given trlx_ppo_loss_from_hidden_workspace_bytes, the *_ex drop-in pair with a saved region — else 1), 1 the
// recompute plan (k_lmloss_dw: Sᵀ recomputed, 4 MFMA passes), 4 the saved-P plan (k_lmloss_dwp:
// 3 passes).  The round-5 H-sliced forms (2, 3) and the 32x32 pair forward (lmloss_fwd = 1) were
// measured slower and removed (git history keeps them; DESIGN.md §3 lists the measurements).
static TuneKnob g_ll_dw{0};
// tuning "lmloss_dwp_form": the saved-P dW kernel's blocking, vocab rows per wave 16·RW x hidden
// parts (workgroups per vocab block): 0 auto (= 2), 1 = RW 1 / whole H, 2 = RW 2 / H halves
static TuneKnob g_ll_form{0};

int lmloss_set_tuning(const char* key, int64_t value, bool* handled) {
    const bool sp = key && !__builtin_strcmp(key, "lmloss_splits");
    const bool ts = key && !__builtin_strcmp(key, "lmloss_dw_tsplit");
    const bool fw = key && !__builtin_strcmp(key, "lmloss_fwd");
    const bool dwk = key && !__builtin_strcmp(key, "lmloss_dw");
    const bool rwk = key && !__builtin_strcmp(key, "lmloss_dwp_form");
    *handled = sp || ts || fw || dwk || rwk;
    if (rwk) {
        TRLX_REQUIRE(value >= 0 && value <= 2, TRLX_ERR_ARG, "lmloss_dwp_form: 0 auto, 1, 2");
        g_ll_form = int(value);
        return TRLX_OK;
    }
    if (fw) {  // one forward form is built: the 16x16x32 one (0 / 2 select it)
        TRLX_REQUIRE(value == 0 || value == 2, TRLX_ERR_ARG,
                     "lmloss_fwd: only the 16x16x32 form (0 auto, 2) is built; forms 1, 3, 4 were removed");
        return TRLX_OK;
    }
    if (dwk) {
        TRLX_REQUIRE(value == 0 || value == 1 || value == 4, TRLX_ERR_ARG,
                     "lmloss_dw: 0 auto, 1 recompute plan, 4 saved P (the H-sliced forms 2, 3 were removed)");
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
    uint16_t* hq;
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

// The saved-P dW forms (tuning "lmloss_dwp_form"; 0 = the default, kLLDwpForm): vocab rows per
// block (64·RW), hidden parts (workgroups per block) and workgroups per CU.  The recompute plan's
// k_lmloss_dw is form 1's shape (64 rows x H).
// Measured and dropped (round 6, profiles/r06f_dwp_forms_*.jsonl, interleaved, whole update): RW 2
// with 256 hidden columns a workgroup and two workgroups per CU (+3 % C2, +4 % C3), RW 4 with 256
// columns (+1 % / +2 %), and the hidden parts of a block back to back on one XCD (±0.3 %).
struct LlDwForm {
    int rw, hsp, vpw;
};
constexpr int kLLDwpForm = 2;
static LlDwForm ll_dw_form(int f, int64_t H) {
    (void)H;
    return f == 1 ? LlDwForm{1, 1, 64} : LlDwForm{2, 2, 128};
}

// dW grid plan: whole rounds of workgroups own a vocab block each; the blocks of the last,
// partial round are split over the tokens so that round is (nearly) full instead of a tail of
// a few long workgroups (C2: 786 blocks on 256 CUs = 3 rounds + 18 blocks, the 18 split 14 ways).
struct LlDwPlan {
    int full, tsplit, nblk;  // workgroups = full + nblk·tsplit
};
// parts: workgroups per vocab block (the saved-P forms' hidden parts)
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
// the saved P tiles (⌈V/64⌉ x 2⌈N/64⌉ x 4 KB: 0.62 GB at C2) and the per-(split, token) records
static size_t ll_pbuf_bytes(int64_t N, int64_t V) { return size_t((V + 63) / 64) * ll_pntt(N) * 4096; }
static size_t ll_hq_bytes(int64_t N, int64_t H) { return size_t(kLLMaxSplits) * N * H * 2; }
static size_t ll_erec_bytes(int64_t N) { return size_t(kLLMaxSplits) * N * 4; }
// the dwp kernel addresses hq rows through a 32-bit buffer resource (ll_check's bound)
static bool ll_hq_fits(int64_t N, int64_t H) { return int64_t(ll_hq_bytes(N, H)) < kLLMaxSpan; }

// Workspace carve-up for N tokens (dwpart: the split blocks' fp32 partials).
//   fwd:  the forward's partials (O, (m, l)) — false for the backward's own workspace
//   pbuf: the saved P tiles (the PPO entries' saved-P plan)
//   hq:   the token rows scaled per split that the dwp kernel streams (the PPO saved-P plan,
//         every backward: 8·N·H·2 B, 75 MB at C2)
static size_t ll_carve(void* base, int64_t N, int64_t H, int64_t V, LlWs* w, bool fwd, bool pbuf, bool hq) {
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
    t.flags = reinterpret_cast<int*>(take(size_t((N + kLLRows - 1) / kLLRows) * kLLMaxSplits * 4 * 4));  // 4 waves a workgroup
    size_t dwp = 0;  // the largest token-split partial buffer over the dW forms
    for (int f = 1; f <= 2; ++f) {
        const LlDwForm fm = ll_dw_form(f, H);
        const LlDwPlan d = ll_dw_plan(V, fm.vpw, fm.hsp);
        dwp = std::max(dwp, size_t(d.nblk) * d.tsplit * fm.vpw);
    }
    t.dwpart = reinterpret_cast<float*>(take(dwp * H * 4));
    t.pbuf = reinterpret_cast<uint16_t*>(take(pbuf ? ll_pbuf_bytes(N, V) : 0));
    t.hq = reinterpret_cast<uint16_t*>(take(hq ? ll_hq_bytes(N, H) : 0));
    if (w) *w = t;
    return off;
}
// The drop-in pair's saved region (trlx_lmhead_logprobs_fwd_ex -> _bwd_ex): the P tiles (label
// entries patched) and the per-(split, token) scales e', alive from the forward to the backward
// (the forward's O partials are not).
static size_t ll_saved_carve(void* base, int64_t N, int64_t V, uint16_t** pbuf, float** erec) {
    char* p = static_cast<char*>(base);
    const size_t pb = ll_align(ll_pbuf_bytes(N, V));
    if (pbuf) *pbuf = reinterpret_cast<uint16_t*>(p);
    if (erec) *erec = reinterpret_cast<float*>(p ? p + pb : nullptr);
    return pb + ll_align(ll_erec_bytes(N));
}

static int ll_check(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N, int64_t H,
                    int64_t V) {
    TRLX_REQUIRE(hidden && weight, TRLX_ERR_ARG, "NULL hidden / weight");
    TRLX_REQUIRE(N > 0 && V > 0 && N < (int64_t(1) << 31) && V < (int64_t(1) << 31), TRLX_ERR_SHAPE,
                 "bad shape N=%lld V=%lld", (long long)N, (long long)V);
    TRLX_REQUIRE(H == 512 || H == 768, TRLX_ERR_SHAPE,
                 "fused lm_head loss: hidden size %lld not built (512, 768: a wave's h / W fragments and its "
                 "O / dW accumulators over the whole H must fit its 512 registers)", (long long)H);
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
template <class G>
static int ll_launch_fwd(const LmLossArgs& a, hipStream_t s) {
    const int64_t ntb = (a.N + kLLTokBlock - 1) / kLLTokBlock;
    const unsigned grid = unsigned((ntb * a.nsplit + 7) / 8 * 8);
    void (*first)(LmLossArgs) = a.pbuf ? k_lmloss_fwd<G, false, true> : k_lmloss_fwd<G, false, false>;
    void (*restart)(LmLossArgs) = a.pbuf ? k_lmloss_fwd<G, true, true> : k_lmloss_fwd<G, true, false>;
    hipLaunchKernelGGL(first, dim3(grid), dim3(G::kThreads), 0, s, a);
    const int rc = check_launch("k_lmloss_fwd");
    if (rc) return rc;
    hipLaunchKernelGGL(restart, dim3(unsigned(std::min<int64_t>(grid, a.ncu))), dim3(G::kThreads), 0, s, a);
    return check_launch("k_lmloss_fwd restart");
}
template <class G>
static int ll_launch_dw(const LmLossArgs& a, hipStream_t s) {
    const dim3 grid(unsigned(a.dw_full + a.dw_nblk * a.tsplit));
    if (a.pbuf) {
        // HSP workgroups per vocab block
        const unsigned gx = grid.x * unsigned(a.dw_hsp);
        if (a.dw_hsp == 1)
            hipLaunchKernelGGL((k_lmloss_dwp<G, 1, 1>), dim3(gx), dim3(G::kThreads), 0, s, a);
        else
            hipLaunchKernelGGL((k_lmloss_dwp<G, 2, 2>), dim3(gx), dim3(G::kThreads), 0, s, a);
        return check_launch("k_lmloss_dwp");
    }
    hipLaunchKernelGGL(k_lmloss_dw<G>, grid, dim3(G::kThreads), 0, s, a);
    return check_launch("k_lmloss_dw");
}
static int ll_fwd(const LmLossArgs& a, hipStream_t s) {
    return a.H == 512 ? ll_launch_fwd<LlG512>(a, s) : ll_launch_fwd<LlG768>(a, s);
}
static int ll_dw(const LmLossArgs& a, hipStream_t s) {
    return a.H == 512 ? ll_launch_dw<LlG512>(a, s) : ll_launch_dw<LlG768>(a, s);
}

// the common part: shapes, workspace, optional compaction from the mask.  savep: the dW pass
// reads saved P (its grid plan); fwd / pbuf / hq: the caller's workspace carve (ll_carve)
static int ll_setup(LmLossArgs& a, const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                    int64_t H, int64_t V, const int64_t* labels, int64_t lb, const int64_t* compact_mask,
                    void* lm_ws, void* dweight, int dw_dtype, int64_t lddw, LlWs& w, hipStream_t s, bool savep,
                    bool fwd, bool pbuf, bool hq) {
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
    const LlDwForm fm = ll_dw_form(savep ? (g_ll_form ? int(g_ll_form) : kLLDwpForm) : 1, H);
    a.dw_vpw = fm.vpw;
    a.dw_hsp = savep ? fm.hsp : 1;
    // split granules of the dW vocab block (>= 4 tiles: the drop-in forward and backward agree
    // whatever the plan; the tuning must not change between them)
    a.sgran = std::max(4, fm.vpw / kLLRows);
    const LlDwPlan dp = ll_dw_plan(V, fm.vpw, a.dw_hsp);
    a.dw_full = dp.full;
    a.tsplit = dp.tsplit;
    a.dw_nblk = dp.nblk;
    ll_carve(lm_ws, N, H, V, &w, fwd, pbuf, hq);
    a.dwpart = w.dwpart;
    a.pbuf = pbuf ? w.pbuf : nullptr;
    a.pntt = ll_pntt(N);
    a.hq = hq ? w.hq : nullptr;
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
    return int64_t(ll_carve(nullptr, N, H, V, nullptr, true, false, false));
}

extern "C" int64_t trlx_lmhead_loss_bwd_workspace_bytes(int64_t N, int64_t H, int64_t V) {
    return int64_t(ll_carve(nullptr, N, H, V, nullptr, false, false, true));
}

extern "C" int64_t trlx_ppo_loss_from_hidden_workspace_bytes(int64_t N, int64_t H, int64_t V) {
    return int64_t(ll_carve(nullptr, N, H, V, nullptr, true, true, true));
}

extern "C" int64_t trlx_lmhead_savep_bytes(int64_t N, int64_t H, int64_t V) {
    (void)H;
    return int64_t(ll_saved_carve(nullptr, N, V, nullptr, nullptr));
}

// The saved-P plan runs when the tuning allows it and the caller's workspace holds the P tiles.
static bool ll_savep_plan(int64_t N, int64_t H, int64_t V, int64_t lm_bytes) {
    return (g_ll_dw == 0 || g_ll_dw == 4) && ll_hq_fits(N, H) &&
           lm_bytes >= int64_t(ll_carve(nullptr, N, H, V, nullptr, true, true, true));
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
    TRLX_REQUIRE(lm_bytes >= int64_t(ll_carve(nullptr, N, H, V, nullptr, true, false, false)), TRLX_ERR_ARG,
                 "lm_workspace of %lld bytes: below trlx_lmhead_loss_workspace_bytes(%lld, %lld, %lld)",
                 (long long)lm_bytes, (long long)N, (long long)H, (long long)V);
    const bool savep = ll_savep_plan(N, H, V, lm_bytes);
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, 1, mask, lm_workspace, dweight, dw_dtype, lddw, w,
                      s, savep, true, savep, savep);
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

// The drop-in autograd pair (lm_head.py): forward -> lp, lse, E; backward -> dh, dW.  The
// *_ex forms keep the forward's bf16 P tiles in the caller's `saved` region
// (trlx_lmhead_savep_bytes) so the backward's dW pass reads them back (k_lmloss_dwp, 3 MFMA
// passes in all) instead of recomputing S (k_lmloss_dw, 4).
static int ll_dropin_fwd(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N, int64_t H,
                         int64_t V, const int64_t* labels, int64_t lb, const int64_t* mask, void* lp_out, int lp_dtype,
                         float* lse_out, float* e_out, void* lm_workspace, void* saved, hipStream_t s) {
    if (N == 0) return TRLX_OK;
    LmLossArgs a = {};
    LlWs w;
    TRLX_REQUIRE(lp_out && lse_out && e_out, TRLX_ERR_ARG, "NULL lp / lse / E output");
    TRLX_REQUIRE(lp_dtype == TRLX_F32 || lp_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "lp dtype");
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, lb, mask, lm_workspace, nullptr, TRLX_F32, H,
                      w, s, saved != nullptr, true, false, false);
    if (rc) return rc;
    if (saved) ll_saved_carve(saved, N, V, &a.pbuf, &a.erec);  // the forward stores P; the combine e' and the label patch
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

static int ll_dropin_bwd(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N, int64_t H,
                         int64_t V, const int64_t* labels, int64_t lb, const int64_t* mask, const void* grad,
                         int grad_dtype, const float* lse, const float* e, void* dhidden, int64_t lddh, int dh_dtype,
                         void* dweight, int dw_dtype, int64_t lddw, void* lm_workspace, const void* saved,
                         hipStream_t s) {
    if (N == 0) return TRLX_OK;
    LmLossArgs a = {};
    LlWs w;
    TRLX_REQUIRE(grad && lse && e, TRLX_ERR_ARG, "NULL grad / lse / E");
    TRLX_REQUIRE(dhidden || dweight, TRLX_ERR_ARG, "neither dhidden nor dweight requested");
    TRLX_REQUIRE(grad_dtype == TRLX_F32 || grad_dtype == TRLX_BF16, TRLX_ERR_DTYPE, "grad dtype");
    TRLX_REQUIRE(dh_dtype == TRLX_BF16 || dh_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dhidden dtype");
    TRLX_REQUIRE(dw_dtype == TRLX_BF16 || dw_dtype == TRLX_F32, TRLX_ERR_DTYPE, "dweight dtype");
    TRLX_REQUIRE(lddh % 4 == 0 && lddh >= H && lddw >= H, TRLX_ERR_STRIDE, "gradient row strides");
    // the saved-P dW pass where the forward kept P (and the scaled rows fit the 2-GB addressing);
    // else the recompute plan, which needs nothing from the forward but lse and E
    const bool savep = saved != nullptr && dweight != nullptr && ll_hq_fits(N, H) && g_ll_dw != 1;
    // the forward's compaction again (launch_order is a stable, deterministic order: the same
    // compact token indices as the forward's records)
    int rc = ll_setup(a, hidden, ldh, weight, ldw, N, H, V, labels, lb, mask, lm_workspace, dweight, dw_dtype, lddw,
                      w, s, savep, false, false, true);
    if (rc) return rc;
    if (savep) {  // the forward's P and e' in; the scaled h rows (w.hq) out
        ll_saved_carve(const_cast<void*>(saved), N, V, &a.pbuf, &a.erec);
    } else {
        a.hq = nullptr;
    }
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

extern "C" int trlx_lmhead_logprobs_fwd_saved(const void* hidden, int64_t ldh, const void* weight, int64_t ldw,
                                              int64_t N, int64_t H, int64_t V, const int64_t* labels, int64_t lb,
                                              void* lp_out, int lp_dtype, float* lse_out, float* e_out,
                                              void* lm_workspace, void* stream) {
    return ll_dropin_fwd(hidden, ldh, weight, ldw, N, H, V, labels, lb, nullptr, lp_out, lp_dtype, lse_out, e_out,
                         lm_workspace, nullptr, (hipStream_t)stream);
}

extern "C" int trlx_lmhead_logprobs_bwd(const void* hidden, int64_t ldh, const void* weight, int64_t ldw, int64_t N,
                                        int64_t H, int64_t V, const int64_t* labels, int64_t lb, const void* grad,
                                        int grad_dtype, const float* lse, const float* e, void* dhidden, int64_t lddh,
                                        int dh_dtype, void* dweight, int dw_dtype, int64_t lddw, void* lm_workspace,
                                        void* stream) {
    return ll_dropin_bwd(hidden, ldh, weight, ldw, N, H, V, labels, lb, nullptr, grad, grad_dtype, lse, e, dhidden,
                         lddh, dh_dtype, dweight, dw_dtype, lddw, lm_workspace, nullptr, (hipStream_t)stream);
}

extern "C" int trlx_lmhead_logprobs_fwd_ex(const void* hidden, int64_t ldh, const void* weight, int64_t ldw,
                                           int64_t N, int64_t H, int64_t V, const int64_t* labels, int64_t lb,
                                           const int64_t* mask, void* lp_out, int lp_dtype, float* lse_out,
                                           float* e_out, void* lm_workspace, void* saved, void* stream) {
    return ll_dropin_fwd(hidden, ldh, weight, ldw, N, H, V, labels, lb, mask, lp_out, lp_dtype, lse_out, e_out,
                         lm_workspace, saved, (hipStream_t)stream);
}

extern "C" int trlx_lmhead_logprobs_bwd_ex(const void* hidden, int64_t ldh, const void* weight, int64_t ldw,
                                           int64_t N, int64_t H, int64_t V, const int64_t* labels, int64_t lb,
                                           const int64_t* mask, const void* grad, int grad_dtype, const float* lse,
                                           const float* e, void* dhidden, int64_t lddh, int dh_dtype, void* dweight,
                                           int dw_dtype, int64_t lddw, void* lm_workspace, const void* saved,
                                           void* stream) {
    return ll_dropin_bwd(hidden, ldh, weight, ldw, N, H, V, labels, lb, mask, grad, grad_dtype, lse, e, dhidden, lddh,
                         dh_dtype, dweight, dw_dtype, lddw, lm_workspace, saved, (hipStream_t)stream);
}

#if LL_STAMP
extern "C" int trlx_debug_ll_stamps(void* dst, int64_t n) {
    return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_ll_stamps), size_t(n) * 8) == hipSuccess ? 0 : 1;
}
#endif
