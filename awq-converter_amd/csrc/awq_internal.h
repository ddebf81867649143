// awq_internal.h — shared host/device definitions of libawq_hip.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/awq_hip.h"
#include "awq_diag.h"

namespace awq {

// ---------------------------------------------------------------------------
// Fast-kernel tile geometry (bf16 / fp16, group_size GS in {32, 64, 128, 256}, K % GS == 0).
//
// A tensor [R, K] is a flat sequence of R*G groups of GS elements (G = K / GS).  A
// wave-tile is 2048 elements = 4 KiB of input = S = 2048 / GS group slots (64, 32, 16, 8).
// qzeros packs C = 32/bits consecutive groups of ONE row per word, so a row has
// WPR = ceil(G/C) words.  Two tilings (a wave-tile is <= S groups = one contiguous byte
// range):
//   * byte tiles ("bytes" = 1): when a row's zero points fill whole BYTES of qzeros
//     (8-bit, or 4-bit with G even), tiles are S consecutive flat groups and every
//     tile writes the qzeros bytes of its own groups (byte stores, pad bytes of a row's
//     last word written by the tile holding the row's last group) — full tiles for any
//     such G (GS 128, K = 768: 16 groups per tile, not 12);
//   * word tiles (4-bit with G odd): a tile is WPT consecutive qzeros words, so every
//     word is produced inside one tile:  WPR == 1 (G <= C): WPT = S / G whole rows,
//     else WPT = S / C words (= S groups when every word is full).  S >= C always.
// When G % C == 0 both tilings coincide (S-group tiles of whole words).
// Padded rows (K % gs != 0, K % 8 == 0; the reference zero-pads each row's tail group,
// awq.py:337-339): row tiles — a tile never leaves its row (tiles per row TR = ceil(G / S));
// the loads stop at the row end (the buffer range check returns the padding zeros) and
// every tile owns whole qzeros words (S is a multiple of C).  K % 8 == 0 keeps every
// 8-element lane chunk, packed word and tensor_q store either wholly inside or wholly
// outside the row.
// ---------------------------------------------------------------------------
constexpr int kTileElems = 2048;     // elements per wave-tile (4 loads x 64 lanes x 8)
constexpr int kGroup = 128;          // the benchmark's group size (BASELINE.json)
#ifndef AWQ_WPB
#define AWQ_WPB 1
#endif
// waves (= tiles) per workgroup of the one-wave-per-tile grid.  1 (64-thread workgroups):
// measured best on every large set (r2e, profiles/round2/r2e_kbench_wpb.log: Llama-3-8B
// set 0.778 -> 0.803 of 8 TB/s from 8 -> 1; opt-125m 0.716 -> 0.737) — a finished wave's
// slot is refilled one wave at a time instead of waiting for its workgroup's slowest wave
constexpr int kWavesPerBlock = AWQ_WPB;
// tiles per entry of the host-planned tensor table (include/awq_hip.h AWQ_BLOCK_TILES).
// One-wave workgroups are dealt round-robin over the 8 XCDs, so tile t runs on XCD t % 8;
// an entry covers the 8 tiles of ONE XCD inside a 64-tile window (t0 + 8 j), and the two
// entries of an XCD for windows 2k and 2k + 1 share a 128-B line, so each table line is
// fetched by one XCD's L2 (entries of 8 consecutive tiles were fetched by all 8 L2s:
// +2.3 % HBM reads on the 70B set, profiles/round3/r3k).
constexpr int kTableTiles = AWQ_BLOCK_TILES;
static_assert(AWQ_BLOCK_TILES == 8, "the XCD-interleaved table layout assumes 8 tiles per entry");
__host__ __device__ inline int64_t table_index(int64_t t) {   // entry of tile t
    return (t >> 7) * 16 + (t & 7) * 2 + ((t >> 6) & 1);
}
__host__ __device__ inline int64_t table_first_tile(int64_t b) {   // first tile of entry b
    return (b >> 4) * 128 + (b & 1) * 64 + ((b & 15) >> 1);
}
__host__ __device__ inline int64_t table_entries(int64_t total_tiles) {
    return (total_tiles + 127) / 128 * 16;
}
// One entry of the tensor table per kTableTiles tiles (awq_plan_block_tensor): everything a
// wave needs to issue its tile's loads — the tensor's input, first tile and shape — in one
// 64-B scalar load, so the loads no longer wait for a second, dependent load of the 80-B
// descriptor (which the wave then fetches while its loads are in flight).
struct alignas(16) TableEntry {
    const void* w;        // the tensor's input
    int64_t tile_begin;   // its first tile
    int64_t rows, K;
    int32_t tensor;       // descriptor index; bit 31: the entry's tiles span tensors (slow path)
    int32_t pad[7];
};
static_assert(sizeof(TableEntry) == 64, "table entry");
constexpr int kTableEntryInts = (int)(sizeof(TableEntry) / 4);

// group sizes the streaming kernel is instantiated for (8 elements per lane: GS / 8 lanes
// per group, a power of two between 4 and 32 so the group reductions stay inside DPP rows
// or one permlane16 swap)
__host__ __device__ inline bool fast_group_size(int64_t gs) {
    return gs == 32 || gs == 64 || gs == 128 || gs == 256;
}

struct TensorGeom {
    uint32_t G;    // groups per row
    uint32_t C;    // groups per qzeros word
    uint32_t WPR;  // qzeros words per row
    uint32_t WPT;  // words per tile
    uint32_t words;  // R * WPR
    uint32_t bytes;  // 1 = byte tiles (see above), 0 = word tiles
    uint32_t S;      // group slots per tile
    uint32_t TR;     // padded rows: tiles per row (0 = flat tiling)
};

// pad = false: the caller guarantees K % gs == 0 (kernels built without the row-tile path)
__host__ __device__ inline TensorGeom fast_geom(int64_t R, int64_t K, int bits, int gs, bool pad = true) {
    TensorGeom g;
    g.S = (uint32_t)(kTileElems / gs);
    g.G = (uint32_t)(pad ? (K + gs - 1) / gs : K / gs);
    g.C = 32u / (uint32_t)bits;
    g.WPR = (g.G + g.C - 1) / g.C;
    g.WPT = (g.WPR == 1) ? (g.S / g.G) : (g.S / g.C);
    g.words = (uint32_t)R * g.WPR;
    g.TR = (pad && (K % gs)) ? (g.G + g.S - 1) / g.S : 0u;
    g.bytes = (!g.TR && (bits == 8 || (g.G % 2u) == 0u)) ? 1u : 0u;
    return g;
}

__host__ __device__ inline int64_t fast_tiles(int64_t R, int64_t K, int bits, int gs) {
    if (R <= 0 || K <= 0) return 0;
    TensorGeom g = fast_geom(R, K, bits, gs);
    if (g.TR) return R * (int64_t)g.TR;
    if (g.bytes) return (R * (int64_t)g.G + g.S - 1) / g.S;
    return ((int64_t)g.words + g.WPT - 1) / g.WPT;
}

// first flat group of qzeros word w
__host__ __device__ inline uint32_t word_group(const TensorGeom& g, uint32_t w) {
    uint32_t row = w / g.WPR;
    uint32_t wi = w - row * g.WPR;
    return row * g.G + wi * g.C;
}

// Limits of the fast path: whole groups, or padded rows with K % 8 == 0; flat group
// indices must fit 32 bits.
__host__ __device__ inline bool fast_shape_ok(int64_t R, int64_t K, int64_t gs) {
    if (!fast_group_size(gs) || R <= 0 || K <= 0 || ((K % gs) != 0 && (K % 8) != 0)) return false;
    int64_t G = (K + gs - 1) / gs;
    return R * G < (int64_t)0x7FFFFFFF && R * (G + 1) < (int64_t)0x7FFFFFFF;
}

// ---------------------------------------------------------------------------
// fp16 bits of a NaN scale, as the reference's CPU ops leave them (restated and pinned in
// oracle/awq_oracle.c oracle_nan_scale_f16 against tests/golden/golden_nan.*): torch.min/max
// over >= 2 elements holding a NaN give the all-ones NaN of the compute type, the scale
// arithmetic and the stores of awq.py:202-205, 327/352 and 411 then leave
//   bf16 0x7E00;  fp16 0x7FFF (0xFE00 asym / 0x7E00 sym on the small-tensor path
//   awq.py:130-171, whose scales skip the fp32 buffer);  fp32 / fp64 0xFFFF, and 0xFE00 for a
//   NaN made by inf - inf (an asymmetric all-+inf or all--inf group).
// nan_scale_code packs (group holds a NaN) in the low half and (inf - inf) in the high half.
// One-element groups (n = 1) keep the element's own NaN: nan_scale_one.
// ---------------------------------------------------------------------------
__host__ __device__ inline uint32_t nan_scale_code(int dtype, int sym, bool small) {
    uint32_t in = 0xFFFFu, ar = 0xFE00u;                   // fp32 / fp64
    if (dtype == AWQ_DTYPE_BF16) in = ar = 0x7E00u;
    if (dtype == AWQ_DTYPE_F16) in = ar = !small ? 0x7FFFu : (sym ? 0x7E00u : 0xFE00u);
    return in | (ar << 16);
}
__host__ __device__ inline uint16_t nan_scale_pick(uint32_t code, bool group_nan) {
    return (uint16_t)(group_nan ? code & 0xFFFFu : code >> 16);
}
// n = 1: e = raw bits of the group's element (a NaN, or +-inf for an asymmetric inf - inf)
__host__ __device__ inline uint16_t nan_scale_one(int dtype, int sym, bool small, uint64_t e, bool e_nan) {
    if (dtype == AWQ_DTYPE_BF16) return 0x7E00u;
    if (dtype == AWQ_DTYPE_F16) {
        if (!small) return 0x7FFFu;
        if (sym) return 0x7E00u;
        return e_nan ? (uint16_t)((e & 0x8000u) | 0x7E00u) : (uint16_t)0xFE00u;
    }
    if (!e_nan) return 0xFE00u;
    const bool f64 = dtype == AWQ_DTYPE_F64;
    uint16_t sign = (uint16_t)(f64 ? (e >> 48) & 0x8000u : (e >> 16) & 0x8000u);
    const uint16_t m10 = (uint16_t)(f64 ? (e >> 42) & 0x3FFu : (e >> 13) & 0x3FFu);
    if (sym) sign = 0x8000u;
    return (uint16_t)(sign | 0x7E00u | m10);
}
// dequantize (awq.py:459-539): the fp32 output of a NaN product at in-group position i of a
// group of n = min(L, K - g L) elements — ATen's fp16 -> fp32 copy (awq.py:527/531) widens
// 8-element vectors bit-preservingly (f16 NaN bits h) and converts the last n % 8 one by one,
// which turns any NaN into 0x7FFFFFFF
__host__ __device__ inline uint32_t dq_nan_bits(uint16_t h, int64_t i, int64_t n) {
    if (i >= (n & ~(int64_t)7)) return 0x7FFFFFFFu;
    return ((uint32_t)(h & 0x8000u) << 16) | 0x7F800000u | ((uint32_t)(h & 0x3FFu) << 13);
}

// the calling thread's diagnostics overrides (csrc/awq_diag.h, diagnostics build; all zero = defaults)
#ifdef AWQ_DIAG
const awq_tuning& tuning();   // awq_capi.hip: this thread's awq_set_tuning overrides
#else
// the product build: the measured defaults, compile-time constant (every override folds away)
inline const awq_tuning& tuning() {
    static constexpr awq_tuning kDefaults{};
    return kDefaults;
}
#endif

// launchers (awq_fast.hip / awq_generic.hip).  nan_code: nan_scale_code() of the call.
hipError_t launch_fast(const awq_tensor_desc* descs_dev, const int32_t* block_tensor,
                       const awq_tensor_desc* single, int n, int64_t total_tiles, int dtype, int bits,
                       int symmetric, int group_size, bool padded, hipStream_t stream, uint32_t nan_code,
                       int n_grid = 1, int n_cand = 0, const float* col_scale = nullptr);
// small: the small-tensor path (NaN scale bits, see nan_scale_code)
hipError_t launch_generic(const void* w, int dtype, int64_t rows, int64_t K, int64_t L, int bits,
                          int symmetric, int32_t* tensor_q, uint16_t* scales, int32_t* zeros,
                          int32_t* qweight, int32_t* qzeros, hipStream_t stream, bool small, int n_grid = 1,
                          int n_cand = 0, double* s_exact = nullptr,
                          double* z_exact = nullptr, bool torch_gpu = false);
// x of dtype xdt (AWQ_DTYPE_* incl. I32); first op in d1, second (= out) in d2; flags AWQ_APPLY_*
hipError_t launch_apply(const void* x, int xdt, int64_t rows, int64_t K, int64_t L, const double* scales,
                        const double* zeros, int qmin, int qmax, int mode, int d1, int d2, int flags, void* out,
                        hipStream_t stream);
// any group size <= 512 (fp32: 256), bf16 / fp16 / fp32, any K; rowgroup_gpt() = 0: not eligible
int rowgroup_gpt(int dtype, int64_t K, int64_t L);
hipError_t launch_rowgroup(const void* w, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int symmetric,
                           int32_t* qweight, int32_t* qzeros, uint16_t* scales, int32_t* tensor_q, int32_t* zeros,
                           hipStream_t stream, uint32_t nan_code);
hipError_t launch_selftest(int which, unsigned long long* out, hipStream_t stream);
hipError_t launch_stream_copy(const void* src, void* dst, int64_t bytes, hipStream_t stream);
hipError_t launch_stream_ceiling(const void* src, void* dst, int64_t bytes, hipStream_t stream);
hipError_t launch_dequant_ceiling(const void* words, void* out, int64_t out_bytes, hipStream_t stream);
hipError_t launch_export_gemm(const int32_t* qweight, const int32_t* qzeros, const uint16_t* scales, int64_t N,
                              int64_t K, int64_t group_size, int32_t* qweight_t, int32_t* qzeros_t,
                              uint16_t* scales_t, hipStream_t stream);
hipError_t launch_pack(const int32_t* v, int64_t rows, int64_t n, int bits, int qmin,
                       int32_t* packed, hipStream_t stream);
hipError_t launch_dequant(const int32_t* tensor_q, const int32_t* qweight, const uint16_t* scales,
                          const int32_t* zeros, const int32_t* qzeros, int64_t rows, int64_t K,
                          int64_t L, int bits, int qmin, float* out, hipStream_t stream);

// activation-aware scale search (awq_actsearch.hip)
hipError_t launch_act_stats(const void* x, int dtype, int64_t T, int64_t K, double* work, float* x_mean,
                            float* x_sq, hipStream_t stream);
hipError_t launch_weight_colsum(const void* w, int dtype, int64_t R, int64_t K, int64_t L, float* gmax,
                                double* part, hipStream_t stream);
hipError_t launch_colmean(const double* part, int64_t nblk, int64_t K, double divisor, float* out,
                          hipStream_t stream);
hipError_t launch_scale_table(const float* x_mean, const float* w_mean, int64_t K, int n_grid, float* table,
                              hipStream_t stream);
hipError_t launch_scale_table_ws(const float* x_mean, const float* w_mean, int64_t K, int n_grid, double* work,
                                 float* table, hipStream_t stream);
hipError_t launch_act_losses(const void* w, int dtype, int64_t R, int64_t K, int64_t L, int bits, int symmetric,
                             const float* table, const float* rtable, int n_grid, const float* x_sq, float* part,
                             int64_t stride, hipStream_t stream);
hipError_t launch_recip_table(const float* table, int64_t n, float* rtable, hipStream_t stream);
hipError_t launch_selftest_mquot(unsigned long long* out, hipStream_t stream);
hipError_t launch_act_select(const float* part, int n_grid, int64_t stride, const float* table, int64_t K,
                             double* work, double* losses, int32_t* best, float* s_best, hipStream_t stream);
hipError_t launch_apply_scale(const void* w, int dtype, int64_t R, int64_t K, const float* s, void* out,
                              hipStream_t stream);

}  // namespace awq
