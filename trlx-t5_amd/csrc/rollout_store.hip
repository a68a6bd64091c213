// Device-resident rollout store: the row gather/scatter that replaces
// the reference's `.cpu()` of five tensors per chunk, per-sample PPORLElement lists and the
// pad_sequence collate (ppo_orchestrator.py:169-187, ppo_pipeline.py:22-68).
//
// The store keeps each field as a padded columnar [capacity, W] buffer in HBM (queries
// right-aligned = left-padded, responses / logprobs / values / rewards left-aligned =
// right-padded, the pad already in place), so both pushing a generation batch and
// collating a training batch are one launch of k_rows_copy: up to kMaxFields fields, each
//   dst[drow(j), dcol0 + c] = src[srow(j), scol0 + c]     j < rows, c < cols
// with srow / drow either contiguous (row0 + j) or an int64 index vector.  Elements are 2,
// 4 or 8 bytes; the copy moves 4- or 8-byte words when the field's byte offsets allow and
// single elements otherwise.  Pure data movement: HBM / latency bound, no arithmetic.
#include "common.h"

namespace trlx {

constexpr int kMaxFields = 8;

struct RowsField {
    const char* src;
    char* dst;
    int64_t src_ld, dst_ld;          // row strides in elements
    int64_t src_col0, dst_col0, cols;
    int esize;                        // bytes per element: 2, 4, 8
};

struct RowsCopyArgs {
    RowsField f[kMaxFields];
    int nfields;
    int64_t rows;
    const int64_t* src_idx;          // NULL: src_row0 + j
    const int64_t* dst_idx;          // NULL: dst_row0 + j
    int64_t src_row0, dst_row0;
};

// grid.x: row blocks (kRowsPerBlock rows each), grid.y: fields.  One wave per row; lanes
// stride over the row's words.
constexpr int kRowsThreads = 256;
constexpr int kRowsPerBlock = kRowsThreads / kWave;

template <typename W>
__device__ __forceinline__ void copy_row(const RowsField& f, int64_t sr, int64_t dr, int lane) {
    const int64_t wpe = int64_t(sizeof(W)) / f.esize;  // elements per word (>= 1)
    const W* s = reinterpret_cast<const W*>(f.src + (sr * f.src_ld + f.src_col0) * f.esize);
    W* d = reinterpret_cast<W*>(f.dst + (dr * f.dst_ld + f.dst_col0) * f.esize);
    const int64_t nw = f.cols / wpe;
    for (int64_t w = lane; w < nw; w += kWave) d[w] = s[w];
}

__global__ __launch_bounds__(kRowsThreads) void k_rows_copy(RowsCopyArgs a) {
    const int64_t j = int64_t(blockIdx.x) * kRowsPerBlock + threadIdx.x / kWave;
    const int lane = threadIdx.x & (kWave - 1);
    if (j >= a.rows) return;
    const RowsField& f = a.f[blockIdx.y];
    const int64_t sr = a.src_idx ? a.src_idx[j] : a.src_row0 + j;
    const int64_t dr = a.dst_idx ? a.dst_idx[j] : a.dst_row0 + j;
    // widest word that divides every byte offset and the row length of this field
    const int64_t sb = (sr * f.src_ld + f.src_col0) * f.esize, db = (dr * f.dst_ld + f.dst_col0) * f.esize;
    const uintptr_t align = (reinterpret_cast<uintptr_t>(f.src) + sb) | (reinterpret_cast<uintptr_t>(f.dst) + db) |
                            uintptr_t(f.cols * f.esize);
    if ((align & 7) == 0 || f.esize == 8)
        copy_row<uint64_t>(f, sr, dr, lane);
    else if ((align & 3) == 0 || f.esize == 4)
        copy_row<uint32_t>(f, sr, dr, lane);
    else
        copy_row<uint16_t>(f, sr, dr, lane);
}

// decoder_input_ids from the response tokens (shift_tokens_right, accelerate_ppo_model.py:18-25):
//   out[b, 0] = start, out[b, t] = ids[b, t-1] (t >= 1), then every -100 (the label ignore id,
//   the start id included) -> pad.  One thread per element, int64 in and out.
__global__ __launch_bounds__(kRowsThreads) void k_shift_tokens_right(const int64_t* ids, int64_t B, int64_t T,
                                                                    int64_t ld, int64_t pad, int64_t start,
                                                                    int64_t* out, int64_t out_ld) {
    const int64_t i = int64_t(blockIdx.x) * kRowsThreads + threadIdx.x;
    if (i >= B * T) return;
    const int64_t b = i / T, t = i - b * T;
    const int64_t v = t == 0 ? start : ids[b * ld + t - 1];
    out[b * out_ld + t] = v == -100 ? pad : v;
}

}  // namespace trlx

using namespace trlx;

extern "C" int trlx_shift_tokens_right(const int64_t* ids, int64_t B, int64_t T, int64_t ld,
                                       int64_t pad_token_id, int64_t decoder_start_token_id, int64_t* out,
                                       int64_t out_ld, void* stream) {
    TRLX_REQUIRE(B >= 0 && T >= 1 && ld >= T && out_ld >= T, TRLX_ERR_SHAPE,
                 "shift_tokens_right: bad shape B=%lld T=%lld (T >= 1, row strides >= T)", (long long)B,
                 (long long)T);
    TRLX_REQUIRE(B * T < (int64_t(1) << 31) * kRowsThreads, TRLX_ERR_SHAPE, "shift_tokens_right: too many tokens");
    if (B == 0) return TRLX_OK;
    TRLX_REQUIRE(ids && out, TRLX_ERR_ARG, "NULL argument to trlx_shift_tokens_right");
    TRLX_REQUIRE(ids != out, TRLX_ERR_ARG, "shift_tokens_right: in-place call (out aliases ids)");
    const unsigned grid = unsigned((B * T + kRowsThreads - 1) / kRowsThreads);
    hipLaunchKernelGGL(k_shift_tokens_right, dim3(grid), dim3(kRowsThreads), 0, (hipStream_t)stream, ids, B, T,
                       ld, pad_token_id, decoder_start_token_id, out, out_ld);
    return check_launch("k_shift_tokens_right");
}

extern "C" int trlx_rows_copy(int nfields, const void* const* src, void* const* dst, const int64_t* src_ld,
                              const int64_t* dst_ld, const int64_t* src_col0, const int64_t* dst_col0,
                              const int64_t* cols, const int* esize, int64_t rows, const int64_t* src_idx,
                              int64_t src_row0, const int64_t* dst_idx, int64_t dst_row0, void* stream) {
    TRLX_REQUIRE(nfields >= 1 && nfields <= kMaxFields, TRLX_ERR_ARG, "nfields must be 1..%d", kMaxFields);
    TRLX_REQUIRE(rows >= 0 && rows < (int64_t(1) << 31) * kRowsPerBlock, TRLX_ERR_SHAPE, "bad row count");
    if (rows == 0) return TRLX_OK;
    RowsCopyArgs a = {};
    a.nfields = nfields;
    a.rows = rows;
    a.src_idx = src_idx;
    a.dst_idx = dst_idx;
    a.src_row0 = src_row0;
    a.dst_row0 = dst_row0;
    for (int i = 0; i < nfields; ++i) {
        TRLX_REQUIRE(src[i] && dst[i], TRLX_ERR_ARG, "NULL field %d", i);
        TRLX_REQUIRE(esize[i] == 2 || esize[i] == 4 || esize[i] == 8, TRLX_ERR_DTYPE, "element size %d", esize[i]);
        TRLX_REQUIRE(cols[i] >= 0 && src_col0[i] >= 0 && dst_col0[i] >= 0, TRLX_ERR_SHAPE, "bad columns");
        a.f[i] = {static_cast<const char*>(src[i]), static_cast<char*>(dst[i]), src_ld[i], dst_ld[i], src_col0[i],
                  dst_col0[i], cols[i], esize[i]};
    }
    const dim3 grid(unsigned((rows + kRowsPerBlock - 1) / kRowsPerBlock), unsigned(nfields));
    hipLaunchKernelGGL(k_rows_copy, grid, dim3(kRowsThreads), 0, (hipStream_t)stream, a);
    return check_launch("k_rows_copy");
}
