// awq_fast.hip — streaming group quantizer for bf16 / fp16 / fp32 weights, group_size
// 32, 64, 128 or 256 (gfx950).
//
// Replaces the per-group Python double loop of the reference
// (src/awq_quantizer/quantization/awq.py:286-374 -> _compute_scale_zp_for_group :173-213
// -> _quantize_tensor :215-250) with one HBM pass: read the weights once, write packed
// qweight/qzeros + fp16 scales (and, in parity mode, the reference's unpacked int32
// tensor_q / zero_points).
//
// Mapping (HBM-bound, no MFMA; described for bf16, GS 128 — the benchmark — with the
// general rule in brackets):
//   * one wave = one tile = 2048 elements = 4 KiB of bf16 [2048 / GS group slots]; lane l
//     holds elements 512 j + 8 l .. + 7 of load j, one 16-B buffer_load_dwordx4 [two for
//     fp32], so a group spans 16 lanes [L = GS / 8] and lane-row rho holds groups 4j + rho;
//   * the grid has one wave per tile (non-persistent): the hardware dispatcher hands a
//     finished wave's slot to the next workgroup, which balances the load across CUs.  A
//     persistent grid (waves walking tiles) lost ~20 % to the dispatcher's age priority:
//     the youngest workgroups of every CU ran last and alone (profiles/r24-r27);
//   * per-group min/max from the raw bits (signed / unsigned integer max), reduced over
//     the group's lanes with DPP-fused v_max [plus one v_permlane16_swap at GS 256]; NaN
//     is detected from the bits;
//   * the scale / zero point of the tile's groups are computed ONCE per lane set (lane c of
//     a group owns the group of load c & 3), with the reference's per-op rounding, then
//     broadcast to the group's lanes with one DPP quad_perm per parameter;
//   * per element: RN_bf16(x * RN_f32(1/s)) == RN_bf16(x / s) for every bf16 x and every
//     bf16 s >= RN_bf16(1e-10) (verified exhaustively: oracle/verify_recip.c), so one
//     multiply replaces the division; RNE to bf16 is one v_cvt_pk_bf16_f32 with a zero
//     low half (the dword IS the rounded f32); + z, round-half-even, clamp, and
//     v_cvt_pk_u8_f32 packs nibble pairs / bytes [fp16: plain or Markstein quotient;
//     fp32: the IEEE division];
//   * each lane emits one packed int32 per load (4-bit), staged in LDS into one 16-B store
//     per lane;
//   * buffer descriptors are based at the tile start with the tile's byte length, so
//     slots past the tile end read zeros and their stores are dropped by the hardware
//     range check (no per-lane masks, no OOB access, tensors > 4 GB are fine).
// Ragged launches: one grid over the tiles of many tensors (descriptor table in HBM); a
// wave finds its tensor from a host-planned per-workgroup table (or, without it, a
// 64-lane ballot search of the descriptors).
#include "awq_quant.h"

namespace awq {
namespace {

struct TileCtx {
    int32_t* qweight;    // tensor bases of the outputs (nullptr = not wanted)
    int32_t* qzeros;
    uint16_t* scales;
    int32_t* tensor_q;
    int32_t* zeros;
    uint32_t start;      // flat group index of the tile's first group
    uint32_t ng;         // groups in the tile (<= S = 2048 / GS)
    uint32_t w0, nw;     // qzeros word range
    uint32_t G, WPR;     // geometry (see awq_internal.h)
    uint32_t r0, g0;     // row / group-in-row of the tile's first group
    uint32_t bytes;      // byte tiles (qzeros written byte-wise) vs word tiles
    uint64_t el_off;     // first input / tensor_q element of the tile
    uint32_t valid;      // elements of the tile inside the tensor (padded rows: inside the row)
    uint64_t qw_off;     // first qweight word of the tile
    uint32_t qw_n;       // qweight words of the tile
};

template <int BITS, int GS, bool PAD>
__device__ __forceinline__ TileCtx make_ctx(const awq_tensor_desc& d, uint32_t tile) {
    constexpr uint32_t S = kTileElems / GS;
    const TensorGeom g = fast_geom(d.rows, d.K, BITS, GS, PAD);
    constexpr uint32_t WPG = GS * BITS / 32;   // qweight words per group
    TileCtx c;
    c.bytes = g.bytes;
    if (g.TR) {                                // padded rows: row tiles
        const uint32_t r = tile / g.TR;
        c.r0 = r;
        c.g0 = (tile - r * g.TR) * S;
        c.ng = min(S, g.G - c.g0);
        c.start = r * g.G + c.g0;
        c.w0 = r * g.WPR + c.g0 / g.C;
        c.nw = (c.ng + g.C - 1) / g.C;
        c.el_off = (uint64_t)r * (uint64_t)d.K + (uint64_t)c.g0 * GS;
        c.valid = (uint32_t)min((int64_t)c.ng * GS, d.K - (int64_t)c.g0 * GS);
        c.qw_off = (uint64_t)r * (uint64_t)(d.K * BITS / 32) + (uint64_t)c.g0 * WPG;
        c.qw_n = c.valid * BITS / 32;
    } else if (g.bytes) {
        c.start = tile * S;
        c.ng = min(S, (uint32_t)d.rows * g.G - c.start);
        c.r0 = c.start / g.G;
        c.g0 = c.start - c.r0 * g.G;
        c.w0 = 0;
        c.nw = 0;
    } else {
        const uint32_t w0 = tile * g.WPT;
        const uint32_t w1 = min(w0 + g.WPT, g.words);
        const uint32_t r0 = w0 / g.WPR;
        c.r0 = r0;
        c.g0 = (w0 - r0 * g.WPR) * g.C;
        c.start = r0 * g.G + c.g0;
        const uint32_t end = (w1 == g.words) ? (uint32_t)d.rows * g.G : word_group(g, w1);
        c.ng = end - c.start;
        c.w0 = w0;
        c.nw = w1 - w0;
    }
    if (!g.TR) {
        c.el_off = (uint64_t)c.start * GS;
        c.valid = c.ng * GS;
        c.qw_off = (uint64_t)c.start * WPG;
        c.qw_n = c.ng * WPG;
    }
    c.G = g.G;
    c.WPR = g.WPR;
    c.qweight = d.qweight;
    c.qzeros = d.qzeros;
    c.scales = d.scales;
    c.tensor_q = d.tensor_q;
    c.zeros = d.zeros;
    return c;
}

// first element and element count of a tile (the input range it reads; padded rows stop at
// the row end, the range check supplies the zero padding)
template <int BITS, int GS, bool PAD>
__device__ __forceinline__ void tile_src(int64_t rows, int64_t K, uint32_t tile, uint64_t& el_off, uint32_t& valid) {
    constexpr uint32_t S = kTileElems / GS;
    const TensorGeom g = fast_geom(rows, K, BITS, GS, PAD);
    if (g.TR) {
        const uint32_t r = tile / g.TR;
        const uint32_t g0 = (tile - r * g.TR) * S;
        el_off = (uint64_t)r * (uint64_t)K + (uint64_t)g0 * GS;
        valid = (uint32_t)min((int64_t)S * GS, K - (int64_t)g0 * GS);
        return;
    }
    uint32_t start, ng;
    if (g.bytes) {
        start = tile * S;
        ng = min(S, (uint32_t)rows * g.G - start);
    } else {
        const uint32_t w0 = tile * g.WPT;
        const uint32_t w1 = min(w0 + g.WPT, g.words);
        start = word_group(g, w0);
        const uint32_t end = (w1 == g.words) ? (uint32_t)rows * g.G : word_group(g, w1);
        ng = end - start;
    }
    el_off = (uint64_t)start * GS;
    valid = ng * GS;
}

// 4 x 16-B loads per lane: load j covers the tile's bytes [1 KiB j, 1 KiB (j+1)), lane l
// its 16 B at 16 l — group slot j * (64 / L) + l / L, chunk l % L of that group
// (L = GS / 8).  Slots past the tile end fall outside the descriptor's range and read as
// zero.
// fp32: the same element mapping, each lane's 32 B as two 16-B loads (a pair of
// instructions covers 2 KiB contiguously).
template <typename F, int GS>
__device__ __forceinline__ void load_tile(const char* wp, uint32_t valid, Chunk<F::NW> (&v)[4]) {
    const int lane = threadIdx.x & 63;
    const __amdgpu_buffer_rsrc_t rw = rsrc(wp, valid * (uint32_t)F::kBytes);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int h = 0; h < F::NW; ++h)
            v[j].w[h] = __builtin_amdgcn_raw_buffer_load_b128(
                rw, (uint32_t)(j * 512 * F::kBytes + lane * 8 * F::kBytes + 16 * h), 0, AWQ_LOAD_AUX);
}

// sum over the L lanes of a group, pairwise over adjacent lanes (xor 1, xor 2, then the
// half-row and row mirrors and the row swap pair adjacent blocks): every lane ends with the
// same value, the tree include/awq_hip.h (awq_quantize_search) defines for the clip-search
// error
template <int CTRL>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
template <int L>
__device__ __forceinline__ float grp_sum(float v) {
    v = dpp_add<0xB1>(v);                  // quad_perm [1,0,3,2]
    v = dpp_add<0x4E>(v);                  // quad_perm [2,3,0,1]
    if (L >= 8) v = dpp_add<0x141>(v);     // row_half_mirror
    if (L >= 16) v = dpp_add<0x140>(v);    // row_mirror
    if (L >= 32) {                         // (row 2k) + (row 2k+1) on both rows
        const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                        false, false);
        v = __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
    }
    return v;
}

// The same tree for the 4 groups of this lane's loads at once, each lane keeping only the sum
// of the group it scores (load p = lane & 3, the lane's jj): a reduce-scatter.  Pair sums (xor
// 1) keep the two loads of this lane's parity, quad sums (xor 2) the lane's own load; the
// position-preserving partners lane ^ 4 (two bank-masked row rotates) and lane ^ 8 (row_ror:8)
// then add the quads and halves in the order grp_sum does.  Sums are commutative, so every
// group's total is grp_sum's bits.  11.5 VALU slots for four groups instead of 4 x 4 DPP adds.
template <int L>
__device__ __forceinline__ float grp_sum_scatter(const float (&e)[4]) {
    const int lane = threadIdx.x & 63;
    const bool b0 = lane & 1, b1 = lane & 2;
    const float m01 = b0 ? e[1] : e[0], s01 = b0 ? e[0] : e[1];
    const float m23 = b0 ? e[3] : e[2], s23 = b0 ? e[2] : e[3];
    const float u = m01 + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s01), 0xB1, 0xF, 0xF, true));
    const float w = m23 + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s23), 0xB1, 0xF, 0xF, true));
    const float m = b1 ? w : u, s = b1 ? u : w;
    float t = m + __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, s), 0x4E, 0xF, 0xF, true));
    if (L >= 8) {   // lane ^ 4: quads 1, 3 read lane - 4 (row_ror:4), quads 0, 2 lane + 4 (row_ror:12)
        const int tb = __builtin_bit_cast(int, t);
        int x = __builtin_amdgcn_update_dpp(tb, tb, 0x124, 0xF, 0xA, false);
        x = __builtin_amdgcn_update_dpp(x, tb, 0x12C, 0xF, 0x5, false);
        t = t + __builtin_bit_cast(float, x);
    }
    if (L >= 16) t = dpp_add<0x128>(t);    // lane ^ 8: row_ror:8
    if (L >= 32) {                         // (row 2k) + (row 2k+1) on both rows
        const auto p = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, t), __builtin_bit_cast(unsigned, t),
                                                        false, false);
        t = __builtin_bit_cast(float, (unsigned)p[0]) + __builtin_bit_cast(float, (unsigned)p[1]);
    }
    return t;
}

// AWQ_SEARCH_FMA_MIX = 0: the round-5 error chain (A/B builds, scripts/build_variant.sh)
#ifndef AWQ_SEARCH_FMA_MIX
#define AWQ_SEARCH_FMA_MIX 1
#endif
#ifndef AWQ_SEARCH_S_LATE
#define AWQ_SEARCH_S_LATE 1
#endif
// AWQ_SEARCH_F16_PACKED = 0: fp16 search always through the Markstein f32 chain
#ifndef AWQ_SEARCH_F16_PACKED
#define AWQ_SEARCH_F16_PACKED 1
#endif
// AWQ_SEARCH_BF16_HALF = 0: bf16 search's integer steps in f32 (chunk_err) instead of packed fp16
#ifndef AWQ_SEARCH_BF16_HALF
#define AWQ_SEARCH_BF16_HALF 1
#endif
// AWQ_SEARCH_PK_F32 = 0: the bf16 chain's products and + z as plain f32 ops (compiler's choice)
#ifndef AWQ_SEARCH_PK_F32
#define AWQ_SEARCH_PK_F32 1
#endif
// waves per SIMD the search instances are compiled for (the VGPR budget: 4 -> 128, 5 -> 96, 6 -> 80)
#ifndef AWQ_SEARCH_MIN_WAVES
#define AWQ_SEARCH_MIN_WAVES 4
#endif
// AWQ_SEARCH_SCATTER = 0: per-load group sums (grp_sum) and per-load special-scale ballots
#ifndef AWQ_SEARCH_SCATTER
#define AWQ_SEARCH_SCATTER 1
#endif
// Squared error of this lane's 8-element chunk of a group for one candidate (r, z, s) —
// quantize (awq.py:245-248), dequantize the reference's way (fp16(fp16(q - z) * fp16(s)),
// awq.py:459-539), (x - dq)^2 summed in element order.  `special`: the candidate's scale
// is 0 / inf / NaN (exact division, NaN-propagating clamp).
template <typename F, int BITS, bool SYM>
__device__ __forceinline__ float chunk_err(const Chunk<F::NW>& v, float r, float z, float s, float sh, bool special) {
    constexpr float QMIN = SYM ? -(float)(1 << (BITS - 1)) : 0.0f;
    constexpr float QMAX = SYM ? (float)((1 << (BITS - 1)) - 1) : (float)((1 << BITS) - 1);
    const float zf = F::as_fmt(z);
    float acc = 0.0f;
#if AWQ_SEARCH_FMA_MIX
    // element pairs: the two fp16 products packed by one v_cvt_pk_f16_f32 (RNE), then x - dq as
    // v_fma_mix_f32(dq_f16, -1, x) on each half — an exact product and one rounding, i.e. the
    // subtraction's bits, with no fp16 -> f32 widening instruction
    typedef _Float16 h2 __attribute__((ext_vector_type(2)));
#pragma unroll
    for (int i = 0; i < 8; i += 2) {
        float xq[2], qq[2];
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const float x = F::elem(v, i + u);
            float q;
            if (__builtin_expect(special, 0)) {
                const float t = F::rn(opaque(x) / s);
                const float rr = __builtin_rintf(SYM ? t : F::rn(t + zf));
                q = __builtin_isnan(rr) ? rr : __builtin_fminf(__builtin_fmaxf(rr, QMIN), QMAX);
            } else {
                const float t = F::quot(x, s, r);
                q = __builtin_fminf(__builtin_fmaxf(__builtin_rintf(SYM ? t : F::rn(t + zf)), QMIN), QMAX);
            }
            xq[u] = x;
            qq[u] = q;
        }
        const h2 dq = {(_Float16)((qq[0] - zf) * sh), (_Float16)((qq[1] - zf) * sh)};
        float d0, d1;
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d0) : "v"(dq), "v"(xq[0]));
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d1) : "v"(dq), "v"(xq[1]));
        acc = acc + d0 * d0;
        acc = acc + d1 * d1;
    }
#else
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float x = F::elem(v, i);
        float q;
        if (__builtin_expect(special, 0)) {
            const float t = F::rn(opaque(x) / s);
            const float rr = __builtin_rintf(SYM ? t : F::rn(t + zf));
            q = __builtin_isnan(rr) ? rr : __builtin_fminf(__builtin_fmaxf(rr, QMIN), QMAX);
        } else {
            const float t = F::quot(x, s, r);
            q = __builtin_fminf(__builtin_fmaxf(__builtin_rintf(SYM ? t : F::rn(t + zf)), QMIN), QMAX);
        }
        const float dq = (float)(_Float16)((q - zf) * sh);
        const float d = x - dq;
        acc = acc + d * d;
    }
#endif
    return acc;
}

// fp16 weights, every group of the wave with a scale < 14 (FmtF16::plain_ok, the common case):
// the same error with the chain kept in packed fp16 — t = RN_f16(RN_f32(x * r)) (the verified
// plain quotient; one rounding straight to fp16 would miss 890 pairs, oracle/verify_recip.c
// f16f), u = RN_f16(t + z), the integer rint(u) as RN_f16(u + 1024) (unit spacing in
// [1024, 2048), 1024 even: ties stay half-even) clamped to [1024 + qmin', 1024 + qmax'],
// q - z = that - (1024 + z) (exact), dq = RN_f16((q - z) * s) (v_pk_mul_f16: one rounding of the
// exact product, the reference's fp16 multiply), x - dq as v_fma_mix_f32 on the two fp16
// operands.  Two elements per packed instruction.
// (search_words packs the per-group fp16 operands once per lane: zs = {z, s}, qz = 1024 + z -
// qmin in both halves; one DPP each instead of per-load conversions)
template <int BITS, bool SYM>
__device__ __forceinline__ void search_words(float z, float s, uint32_t& zs, uint32_t& qzw) {
    const _Float16 zh = (_Float16)z, sh = (_Float16)s;   // exact: an integer <= 255, an fp16 value
    const _Float16 q = SYM ? (_Float16)(1024 + (1 << (BITS - 1))) : (_Float16)1024 + zh;
    zs = __builtin_bit_cast(uint32_t, (h2v){zh, sh});
    qzw = __builtin_bit_cast(uint32_t, (h2v){q, q});
}

template <int BITS, bool SYM>
__device__ __forceinline__ float chunk_err_f16p(const Chunk<1>& v, float r, uint32_t zs, uint32_t qzw) {
    constexpr float QLO = SYM ? -(float)(1 << (BITS - 1)) : 0.0f;
    constexpr float QHI = SYM ? (float)((1 << (BITS - 1)) - 1) : (float)((1 << BITS) - 1);
    constexpr _Float16 OFF = (_Float16)(SYM ? 1024 + (1 << (BITS - 1)) : 1024);   // rounding bias
    constexpr _Float16 HI = (_Float16)(1024.0f + QHI - QLO);
    const h2v zsv = __builtin_bit_cast(h2v, zs);
    const h2v zz = zsv.xx, ss = zsv.yy, off = {OFF, OFF};
    const h2v lo = {(_Float16)1024, (_Float16)1024}, hi = {HI, HI};
    const h2v qz = __builtin_bit_cast(h2v, qzw);
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t w = v.w[0][i];
        const float x0 = FmtF16::lo(w), x1 = FmtF16::hi(w);
#if AWQ_SEARCH_PK_F32
        f2 p = pk_mul(f2{x0, x1}, f2{r, r});     // one v_pk_mul_f32; the barrier keeps it f32-rounded
        asm volatile("" : "+v"(p));
        const h2v t = __builtin_convertvector(p, h2v);                                     // RN_f16(RN_f32(x r))
#else
        const h2v t = __builtin_convertvector((f2){opaque(x0 * r), opaque(x1 * r)}, h2v);   // RN_f16(RN_f32(x r))
#endif
        const h2v u = SYM ? t : t + zz;                                                    // RN_f16(t + z)
        const h2v q = __builtin_elementwise_min(__builtin_elementwise_max(u + off, lo), hi);   // 1024 + q - qmin
        const h2v dq = (q - qz) * ss;                                                      // RN_f16((q - z) s)
        float d0, d1;
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel_hi:[1,0,1]" : "=v"(d0) : "v"(w), "v"(dq));
        asm("v_fma_mix_f32 %0, %1, 1.0, -%2 op_sel:[1,0,1] op_sel_hi:[1,0,1]" : "=v"(d1) : "v"(w), "v"(dq));
        acc = acc + d0 * d0;
        acc = acc + d1 * d1;
    }
    return acc;
}

// bf16 weights: the bf16 steps as in chunk_err (t = RN_bf16(x r), u = RN_bf16(t + z), f32 form),
// then the integer steps in packed fp16: u is exact in fp16 wherever it matters (8 significant
// bits; |u| < 2^-14 rounds to a value whose rint is 0 all the same, |u| > 65504 becomes inf and
// clamps to the bound it would clamp to anyway), rint + clamp as in chunk_err_f16p, and
// dq = RN_f16((q - z) s) by v_pk_mul_f16 (the exact product rounded once, as the f32 product +
// v_cvt_pk_f16_f32 of chunk_err).
// (qs = {1024 + z - qmin, s} in fp16, packed once per lane by search_words_bf16)
template <int BITS, bool SYM>
__device__ __forceinline__ uint32_t search_words_bf16(float z, float sh16) {
    const _Float16 q = SYM ? (_Float16)(1024 + (1 << (BITS - 1))) : (_Float16)1024 + (_Float16)z;
    return __builtin_bit_cast(uint32_t, (h2v){q, (_Float16)sh16});
}

template <int BITS, bool SYM>
__device__ __forceinline__ float chunk_err_bf16h(const Chunk<1>& v, float r, float z, uint32_t qs) {
    constexpr float QLO = SYM ? -(float)(1 << (BITS - 1)) : 0.0f;
    constexpr float QHI = SYM ? (float)((1 << (BITS - 1)) - 1) : (float)((1 << BITS) - 1);
    constexpr _Float16 OFF = (_Float16)(SYM ? 1024 + (1 << (BITS - 1)) : 1024);
    constexpr _Float16 HI = (_Float16)(1024.0f + QHI - QLO);
    const h2v qsv = __builtin_bit_cast(h2v, qs);
    const h2v qz = qsv.xx, ss = qsv.yy, off = {OFF, OFF};
    const h2v lo = {(_Float16)1024, (_Float16)1024}, hi = {HI, HI};
    float acc = 0.0f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t w = v.w[0][i];
        const float x0 = FmtBF16::lo(w), x1 = FmtBF16::hi(w);
#if AWQ_SEARCH_PK_F32
        // the pair's product and + z as one v_pk_mul_f32 / v_pk_add_f32 each (the same IEEE ops;
        // two plain VOP2 ops only cost one slot when they dual-issue, ~11 % of the time here)
        const f2 p = pk_mul(f2{x0, x1}, f2{r, r});
        const float t0 = rn_bf16(p.x), t1 = rn_bf16(p.y);
        const f2 a = SYM ? f2{t0, t1} : pk_add(f2{t0, t1}, f2{z, z});
        const float u0 = SYM ? t0 : rn_bf16(a.x), u1 = SYM ? t1 : rn_bf16(a.y);
#else
        const float t0 = rn_bf16(x0 * r), t1 = rn_bf16(x1 * r);
        const float u0 = SYM ? t0 : rn_bf16(t0 + z), u1 = SYM ? t1 : rn_bf16(t1 + z);
#endif
        const h2v u = __builtin_convertvector((f2){u0, u1}, h2v);
        const h2v q = __builtin_elementwise_min(__builtin_elementwise_max(u + off, lo), hi);
        const h2v dq = (q - qz) * ss;
        float d0, d1;
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(d0) : "v"(dq), "v"(x0));
        asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(d1) : "v"(dq), "v"(x1));
        acc = acc + d0 * d0;
        acc = acc + d1 * d1;
    }
    return acc;
}

// Opt-in clip search (include/awq_hip.h awq_quantize_search) inside the streaming kernel:
// candidates alpha_i = (n_grid - i) / n_grid shrink [mn, mx]; lane (grp, ch) evaluates the
// candidate's parameters for its parameter group (the one in load ch & 3), the L lanes of a
// group score each of its 4 loads' groups (8 elements per lane, grp_sum), and the smallest
// error (ties: the earlier candidate; NaN never wins) picks the group's final [mn, mx].
// RN(v * alpha) as torch evaluates it (fp32 product, then one rounding to the dtype); the
// barrier stops the fp16 product from becoming a single-rounding v_mad_mixlo_f16
template <typename F>
__device__ __forceinline__ float shrink(float v, float al) {
    return F::rn(opaque(v * al));
}

// alpha_i = RN_f32((n_grid - i) / n_grid) from rn = RN(1 / n_grid) and one Markstein correction:
// the IEEE quotient's bits for every n_grid <= 65536 (exhaustive, oracle/verify_recip.c alpha),
// without an IEEE division per candidate; larger grids divide
__device__ __forceinline__ float search_alpha(int n_grid, int i, float rn) {
    const float a = (float)(n_grid - i), nf = (float)n_grid;
    if (__builtin_expect(n_grid > 65536, 0)) return a / nf;
    const float q = a * rn;
    const float r = __builtin_fmaf(-nf, q, a);
    return __builtin_fmaf(r, rn, q);
}

template <typename F, int BITS, bool SYM, int GS>
__device__ __forceinline__ void search_range(const Chunk<F::NW> (&v)[4], float& gmn, float& gmx, bool gnan, int n_grid,
                                          int n_cand) {
    [[maybe_unused]] const int jj = threadIdx.x & 3;
    const float rn = 1.0f / (float)n_grid;
    constexpr bool kLateS = AWQ_SEARCH_S_LATE && std::is_same<F, FmtBF16>::value;
    float best = __builtin_inff();
    int bi = 0;
    for (int i = 0; i < n_cand; ++i) {
        const float al = search_alpha(n_grid, i, rn);
        const GroupParams cp = params_from_range<F, BITS, SYM>(shrink<F>(gmn, al), shrink<F>(gmx, al));
        const float csh = F::dq_scale(cp.s);
#if AWQ_SEARCH_SCATTER
        // one wave-wide test per candidate: any group of the tile with a 0 / inf / NaN scale sends
        // all four loads through the per-lane special-aware chain (equal bits on the other lanes)
        const bool any_special = __builtin_amdgcn_ballot_w64(!F::fast(cp.r)) != 0;
        // fp16: every scale of the wave < 14 -> the packed plain chain (chunk_err_f16p)
        const bool plain16 = AWQ_SEARCH_F16_PACKED && std::is_same<F, FmtF16>::value &&
                             __builtin_amdgcn_ballot_w64(!F::plain_ok(cp.s)) == 0;
        // the packed chains' fp16 operands, once per lane (a few instructions; unused in the
        // waves that take another chain)
        uint32_t w1 = 0, w2 = 0;
        if constexpr (std::is_same<F, FmtF16>::value) search_words<BITS, SYM>(cp.z, csh, w1, w2);
        else if constexpr (std::is_same<F, FmtBF16>::value) w1 = search_words_bf16<BITS, SYM>(cp.z, csh);
        float e[4];
        // per load: the broadcasts, then a wave-uniform choice of chain (one chain's operands
        // live at a time: the search instances stay at 80 / 96 VGPRs)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float rj = bcast_j(j, cp.r);
            if (__builtin_expect(any_special, 0)) {
                e[j] = chunk_err<F, BITS, SYM>(v[j], rj, SYM ? 0.0f : bcast_j(j, cp.z), bcast_j(j, cp.s), bcast_j(j, csh),
                                               !F::fast(rj));
            } else if constexpr (std::is_same<F, FmtF16>::value) {
                if (plain16) e[j] = chunk_err_f16p<BITS, SYM>(v[j], rj, bcast_u(j, w1), bcast_u(j, w2));
                else e[j] = chunk_err<F, BITS, SYM>(v[j], rj, SYM ? 0.0f : bcast_j(j, cp.z), bcast_j(j, cp.s),
                                                    bcast_j(j, csh), false);
            } else if constexpr (std::is_same<F, FmtBF16>::value && AWQ_SEARCH_BF16_HALF) {
                e[j] = chunk_err_bf16h<BITS, SYM>(v[j], rj, SYM ? 0.0f : bcast_j(j, cp.z), bcast_u(j, w1));
            } else {
                e[j] = chunk_err<F, BITS, SYM>(v[j], rj, SYM ? 0.0f : bcast_j(j, cp.z), kLateS ? 0.0f : bcast_j(j, cp.s),
                                               bcast_j(j, csh), false);
            }
        }
        const float ej = grp_sum_scatter<GS / 8>(e);
        if (ej < best) {
            best = ej;
            bi = i;
        }
#else
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const float rj = bcast_j(j, cp.r);
            const float zj = SYM ? 0.0f : bcast_j(j, cp.z);
            const float hj = bcast_j(j, csh);
            const bool special = !F::fast(rj);
            float e;
            // (the scale itself only feeds the exact division of a 0 / inf / NaN scale: broadcast
            //  in that rare wave only)
            if constexpr (kLateS) {
                // bf16: the common path's quotient is x * RN(1/s) (r alone); the scale itself only
                // feeds the exact division of a 0 / inf / NaN scale — broadcast in that rare wave
                if (__builtin_expect(__ballot(special) != 0, 0))
                    e = chunk_err<F, BITS, SYM>(v[j], rj, zj, bcast_j(j, cp.s), hj, special);
                else e = chunk_err<F, BITS, SYM>(v[j], rj, zj, 0.0f, hj, false);
            } else {   // fp16 (Markstein correction) and fp32 (IEEE division) read s on every path
                const float sj = bcast_j(j, cp.s);
                if (__builtin_expect(__ballot(special) != 0, 0))
                    e = chunk_err<F, BITS, SYM>(v[j], rj, zj, sj, hj, special);
                else e = chunk_err<F, BITS, SYM>(v[j], rj, zj, sj, hj, false);
            }
            e = grp_sum<GS / 8>(e);
            if (j == jj && e < best) {
                best = e;
                bi = i;
            }
        }
#endif
    }
    if (!gnan && bi != 0) {
        const float al = search_alpha(n_grid, bi, rn);
        gmn = shrink<F>(gmn, al);
        gmx = shrink<F>(gmx, al);
    }
}

template <typename F, int BITS, bool SYM, bool SEARCH, int GS>
__device__ __forceinline__ void compute_tile(const TileCtx& c, const Chunk<F::NW> (&v)[4], uint32_t* zw, uint32_t* qstage,
                                             int n_grid, int n_cand, uint32_t nan_code) {
    constexpr int QMIN = SYM ? -(1 << (BITS - 1)) : 0;
    constexpr uint32_t C = 32u / BITS;   // groups per qzeros word
    constexpr int L = GS / 8;            // lanes per group (8 elements = 16 B per lane)
    constexpr int GPJ = 64 / L;          // groups per load instruction
    constexpr uint32_t S = 4 * GPJ;      // group slots per tile
    const int lane = threadIdx.x & 63;
    const int grp = lane / L;            // group of this lane inside each load
    const int ch = lane % L;             // 16-B chunk of the group
    const uint32_t ng = c.ng;

    // ---- 1. group min/max (awq.py:192-193) of the 4 groups this lane's group-lanes hold,
    //         from the raw 16-bit patterns: the SIGNED int16 max is the float max whenever
    //         the group has a value with the sign bit clear, and the UNSIGNED max is the
    //         float min (most negative) whenever it has one with the sign bit set; NaNs land
    //         beyond F::kNanS / F::kNanU.  Single-signed groups (rare in weights; LayerNorm
    //         gammas) take an extra unsigned-min reduction in a wave-uniform branch.
    //         Reductions over the group's L lanes: DPP-fused v_max_i32 (grp_max) ----
    int smx[4];
    uint32_t umx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        int sm;
        uint32_t um;
        F::lane_max(v[j], sm, um);
        smx[j] = grp_max<L>(sm);
        umx[j] = grp_max<L>(um);
    }
    uint32_t umn[4] = {0, 0, 0, 0};
    bool one_signed = false;
#pragma unroll
    for (int j = 0; j < 4; ++j) one_signed |= (smx[j] < 0) || (umx[j] < F::kSign);
    if (__builtin_expect(__ballot(one_signed) != 0, 0)) {
#pragma unroll
        for (int j = 0; j < 4; ++j) umn[j] = F::kOnes - grp_max<L>(F::lane_cmax(v[j]));   // unsigned min
    }
    // ---- 2. scale / zero point: lane (grp, ch) computes the group of load ch & 3, i.e.
    //         slot GPJ * (ch & 3) + grp (the L / 4 lanes of a group with equal ch & 3 do the
    //         same work; for GS 32 every lane owns exactly one of the 64 slots) ----
    const int jj = ch & 3;
    int ssel = smx[0];
    uint32_t usel = umx[0], nsel = umn[0];
#pragma unroll
    for (int j = 1; j < 4; ++j)
        if (jj == j) { ssel = smx[j]; usel = umx[j]; nsel = umn[j]; }
    float gmn, gmx;
    bool gnan;
    group_range<F, SYM>(ssel, usel, nsel, gmn, gmx, gnan);
    if (SEARCH && n_cand > 1) search_range<F, BITS, SYM, GS>(v, gmn, gmx, gnan, n_grid, n_cand);
    const GroupParams p = params_from_range<F, BITS, SYM>(gmn, gmx);
    const uint32_t my_slot = GPJ * (uint32_t)jj + (uint32_t)grp;
    // wave-uniform: every group of the tile admits the plain quotient (F::plain_ok)
    const bool plain = F::kHasPlain && __builtin_amdgcn_ballot_w64(!F::plain_ok(p.s)) == 0;

    // ---- 4. quantize + pack the 4 groups of this lane ----
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        // this group's r, z, s from the quad lane with ch & 3 == j, broadcast just in time
        // (short live ranges)
        const float rj = bcast_j(j, p.r);
        const float zj = SYM ? 0.0f : bcast_j(j, p.z);
        const float sj = bcast_j(j, p.s);
        u2v word = plain ? quant8_fast<F, BITS, SYM, true>(v[j], rj, zj, sj)
                         : quant8_fast<F, BITS, SYM, false>(v[j], rj, zj, sj);
        const bool special = !F::fast(rj);         // scale 0 / inf / NaN
        if (__builtin_expect(special, 0)) {
            // (q values stay local to the rare branches: a q array live across them made
            // the compiler zero-initialise 8 registers per j on the common path)
            uint32_t nib[8];
            int32_t qs[8];
            quant8_special<F, BITS, SYM>(v[j], zj, sj, nib, qs);
            if (BITS == 4) {
                uint32_t acc = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) acc |= nib[i] << (4 * i);
                word.x = acc;
            } else {
                word.x = nib[0] | (nib[1] << 8) | (nib[2] << 16) | (nib[3] << 24);
                word.y = nib[4] | (nib[5] << 8) | (nib[6] << 16) | (nib[7] << 24);
            }
        }
        // this lane's 8 elements are tile elements 512 j + 8 lane: packed word 64 j + lane
        if (c.qweight) {
            // staged in the wave's LDS block in output order (the lanes of one j write 64
            // consecutive words), stored below as one 16-B piece per lane
            if (BITS == 4) qstage[64 * j + lane] = word.x;
            else *(u2v*)(qstage + 128 * j + 2 * lane) = word;
        }
        if (c.tensor_q) {   // reference-layout int32 tensor_q (parity mode)
            int32_t q[8];
            if (__builtin_expect(special, 0)) {
                uint32_t nib[8];
                quant8_special<F, BITS, SYM>(v[j], zj, sj, nib, q);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const uint32_t wd = (BITS == 4) ? word.x : (i < 4 ? word.x : word.y);
                    const uint32_t sh = (BITS == 4) ? 4 * i : 8 * (i & 3);
                    q[i] = (int32_t)((wd >> sh) & ((1u << BITS) - 1u)) + QMIN;
                }
            }
            __amdgpu_buffer_rsrc_t rt = rsrc(c.tensor_q + c.el_off, c.valid * 4u);
            u4 lo = {(uint32_t)q[0], (uint32_t)q[1], (uint32_t)q[2], (uint32_t)q[3]};
            u4 hi = {(uint32_t)q[4], (uint32_t)q[5], (uint32_t)q[6], (uint32_t)q[7]};
            __builtin_amdgcn_raw_buffer_store_b128(lo, rt, (uint32_t)((512 * j + 8 * lane) * 4), 0, AWQ_STORE_AUX);
            __builtin_amdgcn_raw_buffer_store_b128(hi, rt, (uint32_t)((512 * j + 8 * lane) * 4 + 16), 0, AWQ_STORE_AUX);
        }
    }
    if (c.qweight) {   // 4-bit: 1 KiB per tile = one dwordx4 per lane; 8-bit: 2 KiB, two
        __amdgpu_buffer_rsrc_t rq = rsrc(c.qweight + c.qw_off, c.qw_n * 4u);
#pragma unroll
        for (int h = 0; h < (BITS == 4 ? 1 : 2); ++h) {
            const u4 w4 = *(const u4*)(qstage + h * 256 + lane * 4);
            __builtin_amdgcn_raw_buffer_store_b128(w4, rq, (uint32_t)(h * 1024 + lane * 16), 0, AWQ_STORE_AUX);
        }
    }
    // ---- 5. per-group scalars out (after the data registers are dead): lanes ch < 4 hold
    //         the S slots (one store each) ----
    if (ch < 4) {
        if (c.scales) {
            __amdgpu_buffer_rsrc_t rs = rsrc(c.scales + c.start, ng * 2u);
            __builtin_amdgcn_raw_buffer_store_b16(f16_bits(p.s, gnan, nan_code), rs, my_slot * 2u, 0, AWQ_SMALL_AUX);
        }
        if (c.zeros) {
            __amdgpu_buffer_rsrc_t rz = rsrc(c.zeros + c.start, ng * 4u);
            int32_t zi = __builtin_isnan(p.z) ? INT32_MIN : (int32_t)p.z;
            __builtin_amdgcn_raw_buffer_store_b32((uint32_t)zi, rz, my_slot * 4u, 0, AWQ_SMALL_AUX);
        }
    }
    // qzeros, byte tiles: each group's field OR-ed into its byte (wave-private LDS), then one
    // lane per qzeros byte stores it (plus the zero pad bytes ending its row's last word)
    if (c.qzeros && c.bytes) {
        constexpr uint32_t GPB = BITS == 4 ? 2u : 1u;        // groups per byte
        if ((uint32_t)lane < S) zw[lane] = 0u;
        if (ch < 4 && my_slot < ng) {
            uint32_t zn = __builtin_isnan(p.z) ? (uint32_t)(0u - (uint32_t)QMIN) : (uint32_t)((int)p.z - QMIN);
            zn &= (1u << BITS) - 1u;
            atomicOr(&zw[my_slot / GPB], zn << (BITS * (my_slot % GPB)));
        }
        const uint32_t nb = ng / GPB;                         // ng and the tile start are even
        if ((uint32_t)lane < nb) {
            uint32_t g = c.g0 + (uint32_t)lane * GPB, r = c.r0;
            if (g >= c.G) {
                const uint32_t k = g / c.G;
                r += k;
                g -= k * c.G;
            }
            const uint32_t row_bytes = c.WPR * 4u;
            __amdgpu_buffer_rsrc_t rz = rsrc(c.qzeros, 0x7FFFFFFFu);
            const uint32_t at = r * row_bytes + g / GPB;
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)zw[lane], rz, at, 0, AWQ_SMALL_AUX);
            if (g + GPB >= c.G) {                               // row's last byte: zero the pad
                for (uint32_t b = g / GPB + 1; b < row_bytes; ++b)
                    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)0, rz, r * row_bytes + b, 0, AWQ_SMALL_AUX);
            }
        }
    }
    // qzeros, word tiles: each slot's field OR-ed into its word (wave-private LDS), then stored
    if (c.qzeros && !c.bytes) {
        if ((uint32_t)lane < S) zw[lane] = 0u;
        if (ch < 4 && my_slot < ng) {
            uint32_t g = c.g0 + my_slot, r = c.r0;
            if (g >= c.G) {                 // slot lies in a later row of the tile
                const uint32_t k = g / c.G;
                r += k;
                g -= k * c.G;
            }
            const uint32_t wi = r * c.WPR + g / C;
            const uint32_t pos = g % C;
            uint32_t zn = __builtin_isnan(p.z) ? (uint32_t)(0u - (uint32_t)QMIN) : (uint32_t)((int)p.z - QMIN);
            zn &= (1u << BITS) - 1u;
            atomicOr(&zw[wi - c.w0], zn << (BITS * pos));
        }
        if ((uint32_t)lane < c.nw) {
            __amdgpu_buffer_rsrc_t rz = rsrc(c.qzeros + c.w0, c.nw * 4u);
            __builtin_amdgcn_raw_buffer_store_b32(zw[lane], rz, (uint32_t)lane * 4u, 0, AWQ_SMALL_AUX);
        }
    }

}

// Index of the tensor owning tile t, searching descs[base..n) (tile_begin ascending,
// descs[base].tile_begin <= t).  64 lanes probe 64 evenly spaced descriptors per round
// and a ballot narrows the range: one dependent load per round, 1 round for <= 64
// candidates, 2 for <= 4096 — instead of a chain of scalar loads through every tiny
// tensor (a model has ~100 1-tile bias tensors next to each other).
[[maybe_unused]] __device__ __forceinline__ int find_tensor(const awq_tensor_desc* __restrict__ descs, int n, int base,
                                           int64_t t) {
    const int lane = threadIdx.x & 63;
    int span = n - base;
    while (span > 1) {
        const int stride = (span + 63) >> 6;
        const int idx = base + lane * stride;
        const bool ok = (idx < base + span) && descs[min(idx, n - 1)].tile_begin <= t;
        const int cnt = __builtin_popcountll(__ballot(ok));   // ok lanes form a prefix
        base += (cnt - 1) * stride;
        span = min(stride, n - base);
    }
    return __builtin_amdgcn_readfirstlane(base);
}

// SCALED (awq_quantize_groups_scaled, the activation-aware search's last step): each loaded
// element times its column's col_scale, rounded to the dtype — awq_apply_input_scale's
// RN(w * s) — applied to the raw chunks in place, so compute_tile quantizes W * diag(s)
// without the scaled copy ever being written.  A non-PAD tile is 2048 consecutive elements
// starting at column col0 of its first row; chunks of 8 never straddle rows (K % 8 == 0).
template <typename F>
__device__ __forceinline__ void scale_chunks(Chunk<F::NW> (&v)[4], const float* __restrict__ cs, uint64_t el_off,
                                             int64_t K) {
    const int lane = threadIdx.x & 63;
    const uint32_t k32 = (uint32_t)K;
    const uint32_t col0 = (uint32_t)(el_off % (uint64_t)K);   // wave-uniform
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t idx = col0 + 512u * j + 8u * lane;
        const uint32_t col = k32 >= 2048u ? (idx >= k32 ? idx - k32 : idx) : idx % k32;
        const float4 a = *(const float4*)(cs + col), b = *(const float4*)(cs + col + 4);
        const float sv[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        uint32_t bits[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float y = F::rn(F::elem(v[j], i) * sv[i]);
            if constexpr (F::NW == 2) bits[i] = __float_as_uint(y);
            else if constexpr (std::is_same<F, FmtF16>::value) bits[i] = __builtin_bit_cast(uint16_t, (_Float16)y);
            else bits[i] = __float_as_uint(y) >> 16;
        }
        if constexpr (F::NW == 2) {
            v[j].w[0] = u4{bits[0], bits[1], bits[2], bits[3]};
            v[j].w[1] = u4{bits[4], bits[5], bits[6], bits[7]};
        } else {
            v[j].w[0] = u4{bits[0] | (bits[1] << 16), bits[2] | (bits[3] << 16), bits[4] | (bits[5] << 16),
                           bits[6] | (bits[7] << 16)};
        }
    }
}

#ifdef AWQ_TRACE
__device__ uint64_t* g_trace = nullptr;
#endif

// One wave per tile.  The grid normally covers every tile once (launch_fast); a smaller
// grid (awq_diag.h max_blocks, tests) makes each wave walk tiles t, t + nwaves, ... with a
// tensor cursor.
template <typename F, int BITS, bool SYM, bool SEARCH, int GS, bool PAD, bool SCALED = false>
__global__ __launch_bounds__(64 * kWavesPerBlock, SEARCH ? AWQ_SEARCH_MIN_WAVES : (F::kWide ? AWQ_MIN_WAVES_WIDE : AWQ_MIN_WAVES))
void awq_fast_kernel(
    // the scalars every wave needs first lead the argument block (they fit the kernarg
    // preload window of a -mllvm -amdgpu-kernarg-preload-count build); the 80-B single-
    // tensor descriptor goes last
    const int32_t* __restrict__ block_tensor, const awq_tensor_desc* __restrict__ descs, int64_t total_tiles,
    int n, int n_grid, int n_cand, uint32_t nan_code, const float* __restrict__ col_scale, awq_tensor_desc single) {
    __shared__ uint32_t zwords[kWavesPerBlock][kTileElems / GS];
    __shared__ __attribute__((aligned(16))) uint32_t qstage_all[kWavesPerBlock][BITS == 4 ? 256 : 512];
    // wave index made provably uniform so tile/tensor bookkeeping and the buffer
    // descriptors live in SGPRs (no waterfall loops around the descriptors)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    if (wave >= total_tiles) return;
    uint32_t* zw = zwords[wid];
    uint32_t* qs = qstage_all[wid];
#ifdef AWQ_TRACE
    // timing-only build: per wave (start, first tile's loads issued, landed, end) in
    // s_memrealtime ticks (100 MHz, chip-wide clock) -> scripts/trace_waves.py
    const uint64_t tr0 = __builtin_amdgcn_s_memrealtime();
    uint64_t tr1 = 0, tr2 = 0;
#endif
    int cur = 0;
    awq_tensor_desc d = single;
    // the current tensor's input, first tile and shape: what the loads need (from the
    // table entry on a wave's first tile, else from the descriptor)
    const void* src_w = single.w;
    int64_t src_tb = single.tile_begin, src_rows = single.rows, src_K = single.K;
    bool need_d = false;   // d not loaded yet (fast table path): fetched after the loads went out
    if (descs != nullptr) {
        bool fast = false;
        if (block_tensor != nullptr) {
            // host-planned entry of the wave's tile group (awq_plan_block_tensor): ONE 64-B
            // scalar load gives the tensor's input and shape; entries whose tiles span
            // tensors (small tensors) step through the descriptors
            const TableEntry* te = (const TableEntry*)block_tensor + table_index(wave);
            const int32_t e = __builtin_amdgcn_readfirstlane(te->tensor);
            cur = e & 0x7FFFFFFF;
            if (e >= 0) {
                fast = true;
                src_w = te->w;
                src_tb = te->tile_begin;
                src_rows = te->rows;
                src_K = te->K;
                need_d = true;
            } else {
                while (cur + 1 < n && descs[cur + 1].tile_begin <= wave) ++cur;
            }
        } else {
            cur = find_tensor(descs, n, 0, wave);
        }
        if (!fast) {
            d = descs[cur];
            src_w = d.w;
            src_tb = d.tile_begin;
            src_rows = d.rows;
            src_K = d.K;
        }
    }
    for (int64_t t = wave; t < total_tiles; t += nwaves) {
        if (descs != nullptr && t != wave && cur + 1 < n && descs[cur + 1].tile_begin <= t) {
            cur = find_tensor(descs, n, cur + 1, t);
            d = descs[cur];
            need_d = false;
            src_w = d.w;
            src_tb = d.tile_begin;
            src_rows = d.rows;
            src_K = d.K;
        }
        // the input range first (no division for byte tiles): the loads go out before the
        // rest of the tile context (row / group divisions) is computed
        const uint32_t tile = (uint32_t)(t - src_tb);
        uint64_t el_off;
        uint32_t valid;
        tile_src<BITS, GS, PAD>(src_rows, src_K, tile, el_off, valid);
        Chunk<F::NW> va[4];
        load_tile<F, GS>((const char*)src_w + el_off * F::kBytes, valid, va);
        if constexpr (SCALED) scale_chunks<F>(va, col_scale, el_off, src_K);
        if (need_d) {   // the descriptor (outputs) while the loads are in flight
            d = descs[cur];
            need_d = false;
        }
#ifdef AWQ_TRACE
        if (tr1 == 0) {
            tr1 = __builtin_amdgcn_s_memrealtime();
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            tr2 = __builtin_amdgcn_s_memrealtime();
        }
#endif
        compute_tile<F, BITS, SYM, SEARCH, GS>(make_ctx<BITS, GS, PAD>(d, tile), va, zw, qs, n_grid, n_cand, nan_code);
    }
#ifdef AWQ_TRACE
    if (g_trace != nullptr && (threadIdx.x & 63) == 0) {
        g_trace[wave * 4 + 0] = tr0;
        g_trace[wave * 4 + 1] = tr1;
        g_trace[wave * 4 + 2] = tr2;
        g_trace[wave * 4 + 3] = __builtin_amdgcn_s_memrealtime();
    }
#endif
}

// Exhaustive self-test of recip_bf16 over every non-negative bf16 bit pattern
// s >= RN_bf16(1e-10) (incl. inf / NaN): counts results that differ bitwise from the
// IEEE division.
__global__ void awq_selftest_recip_kernel(unsigned long long* mismatches) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h >= 0x8000u) return;
    const float s = __uint_as_float(h << 16);
    if (!(s >= __uint_as_float(0x2EDC0000u)) && !__builtin_isnan(s)) return;
    const float a = recip_bf16(s);
    const float b = 1.0f / s;
    if (__float_as_uint(a) != __float_as_uint(b) && !(__builtin_isnan(a) && __builtin_isnan(b)))
        atomicAdd(mismatches, 1ull);
}

// which = 2: recip_f16 over every positive finite fp16 s against the IEEE division (bitwise)
__global__ void awq_selftest_recip16_kernel(unsigned long long* mismatches) {
    const uint32_t h = blockIdx.x * blockDim.x + threadIdx.x;
    if (h == 0 || h >= 0x7C00u) return;
    const float s = (float)__builtin_bit_cast(_Float16, (uint16_t)h);
    const float a = recip_f16(s);
    const float b = 1.0f / s;
    if (__float_as_uint(a) != __float_as_uint(b)) atomicAdd(mismatches, 1ull);
}

}  // namespace

hipError_t launch_fast(const awq_tensor_desc* descs_dev, const int32_t* block_tensor,
                       const awq_tensor_desc* single, int n, int64_t total_tiles, int dtype, int bits,
                       int symmetric, int group_size, bool padded, hipStream_t stream, uint32_t nan_code, int n_grid,
                       int n_cand, const float* col_scale) {
    if (total_tiles <= 0) return hipSuccess;
    // one wave per tile (diagnostics, csrc/awq_diag.h, diagnostics build: tiles_per_wave, max_blocks =
    // grid cap; either makes waves walk several tiles)
    int64_t tpw = 1, max_blocks = INT32_MAX;
    if (tuning().tiles_per_wave > 1) tpw = tuning().tiles_per_wave;
    if (tuning().max_blocks > 0) max_blocks = tuning().max_blocks;
    const int64_t per_block = kWavesPerBlock * tpw;
    int64_t blocks = (total_tiles + per_block - 1) / per_block;
    if (blocks > max_blocks) blocks = max_blocks;
    awq_tensor_desc one{};
    if (single) one = *single;
    // the table is indexed by the wave's first tile: valid for the one-tile-per-wave grid only
    const int32_t* bt = (tpw == 1 && blocks * per_block >= total_tiles) ? block_tensor : nullptr;
    const dim3 grid((unsigned)blocks), block(64 * kWavesPerBlock);
#define AWQ_LAUNCH_GS(Fm, B, S, G)                                                                                  \
    do {                                                                                                            \
        if (col_scale)                                                                                              \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, false, G, false, true>), grid, block, 0, stream, bt,      \
                               descs_dev, total_tiles, n, 1, 0, nan_code, col_scale, one);                          \
        else if (n_cand > 1 && padded)                                                                              \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, true, G, true>), grid, block, 0, stream, bt, descs_dev,   \
                               total_tiles, n, n_grid, n_cand, nan_code, nullptr, one);                             \
        else if (n_cand > 1)                                                                                        \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, true, G, false>), grid, block, 0, stream, bt, descs_dev,  \
                               total_tiles, n, n_grid, n_cand, nan_code, nullptr, one);                             \
        else if (padded)                                                                                            \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, false, G, true>), grid, block, 0, stream, bt, descs_dev,  \
                               total_tiles, n, 1, 0, nan_code, nullptr, one);                                       \
        else                                                                                                        \
            hipLaunchKernelGGL((awq_fast_kernel<Fm, B, S, false, G, false>), grid, block, 0, stream, bt, descs_dev, \
                               total_tiles, n, 1, 0, nan_code, nullptr, one);                                       \
    } while (0)
#define AWQ_LAUNCH(Fm, B, S)                                   \
    switch (group_size) {                                      \
    case 32: AWQ_LAUNCH_GS(Fm, B, S, 32); break;               \
    case 64: AWQ_LAUNCH_GS(Fm, B, S, 64); break;               \
    case 256: AWQ_LAUNCH_GS(Fm, B, S, 256); break;             \
    default: AWQ_LAUNCH_GS(Fm, B, S, 128); break;              \
    }
#define AWQ_LAUNCH_FMT(Fm)                          \
    switch ((bits == 8 ? 2 : 0) + (symmetric ? 1 : 0)) { \
    case 0: AWQ_LAUNCH(Fm, 4, false); break;        \
    case 1: AWQ_LAUNCH(Fm, 4, true); break;         \
    case 2: AWQ_LAUNCH(Fm, 8, false); break;        \
    default: AWQ_LAUNCH(Fm, 8, true); break;        \
    }
    if (!fast_group_size(group_size)) return hipErrorInvalidValue;
    if (col_scale && (padded || n_cand > 1 || descs_dev)) return hipErrorInvalidValue;   // single, unpadded RTN
    if (dtype == AWQ_DTYPE_F16) {
        AWQ_LAUNCH_FMT(FmtF16)
    } else if (dtype == AWQ_DTYPE_F32) {
        AWQ_LAUNCH_FMT(FmtF32)
    } else {
        AWQ_LAUNCH_FMT(FmtBF16)
    }
#undef AWQ_LAUNCH_FMT
#undef AWQ_LAUNCH
#undef AWQ_LAUNCH_GS
    return hipPeekAtLastError();
}

#ifdef AWQ_TRACE
extern "C" int awq_debug_set_trace(void* buf) {
    return hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &buf, sizeof(buf)) == hipSuccess ? 0 : 1;
}
#endif

// Measurement helper (bench.py's copy ceiling): a plain HBM copy with the quantizer's
// memory structure — one wave per 4 KiB, 4 x 16-B nt loads and stores per lane, the same
// one-wave-per-tile grid of 512-thread workgroups.  Read + write bytes = 2 x `bytes`.
__global__ __launch_bounds__(64 * kWavesPerBlock) void awq_stream_copy_kernel(const uint8_t* __restrict__ src,
                                                                             uint8_t* __restrict__ dst,
                                                                             int64_t bytes) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t base = ((int64_t)blockIdx.x * kWavesPerBlock + wid) * 4096;
    if (base >= bytes) return;
    const uint32_t n = (uint32_t)min((int64_t)4096, bytes - base);
    const __amdgpu_buffer_rsrc_t rs = rsrc(src + base, n), rd = rsrc(dst + base, n);
    u4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(j * 1024 + lane * 16), 0, 2);
#pragma unroll
    for (int j = 0; j < 4; ++j) __builtin_amdgcn_raw_buffer_store_b128(v[j], rd, (uint32_t)(j * 1024 + lane * 16), 0, 2);
}

hipError_t launch_stream_copy(const void* src, void* dst, int64_t bytes, hipStream_t stream) {
    if (bytes <= 0) return hipSuccess;
    const int64_t per_block = 4096LL * kWavesPerBlock;
    hipLaunchKernelGGL(awq_stream_copy_kernel, dim3((unsigned)((bytes + per_block - 1) / per_block)),
                       dim3(64 * kWavesPerBlock), 0, stream, (const uint8_t*)src, (uint8_t*)dst, bytes);
    return hipPeekAtLastError();
}

// Measurement helper (bench.py's read-dominant ceiling): the quantizer's memory structure
// and read:write ratio without its arithmetic — one wave per 4 KiB of input (4 x 16-B nt
// loads per lane), the four vectors xor-folded to one, ONE 16-B nt store per lane (1 KiB
// per wave).  Read 4 : write 1, against the packed quantizer's 4096 : 1064 per tile.
__global__ __launch_bounds__(64 * kWavesPerBlock) void awq_stream_ceiling_kernel(const uint8_t* __restrict__ src,
                                                                                uint8_t* __restrict__ dst,
                                                                                int64_t bytes) {
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const int64_t tile = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    const int64_t base = tile * 4096;
    if (base >= bytes) return;
    const uint32_t n = (uint32_t)min((int64_t)4096, bytes - base);
    const __amdgpu_buffer_rsrc_t rs = rsrc(src + base, n), rd = rsrc(dst + tile * 1024, n / 4);
    u4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) v[j] = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(j * 1024 + lane * 16), 0, 2);
    const u4 x = v[0] ^ v[1] ^ v[2] ^ v[3];
    __builtin_amdgcn_raw_buffer_store_b128(x, rd, (uint32_t)(lane * 16), 0, 2);
}

hipError_t launch_stream_ceiling(const void* src, void* dst, int64_t bytes, hipStream_t stream) {
    if (bytes <= 0) return hipSuccess;
    const int64_t per_block = 4096LL * kWavesPerBlock;
    hipLaunchKernelGGL(awq_stream_ceiling_kernel, dim3((unsigned)((bytes + per_block - 1) / per_block)),
                       dim3(64 * kWavesPerBlock), 0, stream, (const uint8_t*)src, (uint8_t*)dst, bytes);
    return hipPeekAtLastError();
}

hipError_t launch_selftest(int which, unsigned long long* out, hipStream_t stream) {
    if (which == 2) {
        hipLaunchKernelGGL(awq_selftest_recip16_kernel, dim3(0x7C00 / 256), dim3(256), 0, stream, out);
        return hipPeekAtLastError();
    }
    if (which != 0) return hipErrorInvalidValue;
    hipLaunchKernelGGL(awq_selftest_recip_kernel, dim3(0x8000 / 256), dim3(256), 0, stream, out);
    return hipPeekAtLastError();
}

}  // namespace awq
