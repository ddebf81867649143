// awq_fast.hip — streaming group quantizer for bf16 weights, group_size 128 (gfx950).
//
// Replaces the per-group Python double loop of the reference
// (src/awq_quantizer/quantization/awq.py:286-374 -> _compute_scale_zp_for_group :173-213
// -> _quantize_tensor :215-250) with one HBM pass: read bf16 once, write packed
// qweight/qzeros + fp16 scales (and, in parity mode, the reference's unpacked int32
// tensor_q / zero_points).
//
// Mapping (HBM-bound, no MFMA):
//   * one group = 128 bf16 = 256 B = 16 lanes x one 16-B buffer_load_dwordx4;
//     a wave covers 4 groups per load, 4 loads in flight per lane = one 16-group tile;
//   * per-group min/max in the integer domain: bf16 bits -> order-preserving int16 key
//     (v_bitop3), v_pk_max_i16/v_pk_min_i16, then max/~min packed in one dword and reduced
//     across the 16-lane DPP row (quad_perm, row_half_mirror, row_mirror) — no LDS;
//     NaN is detected from the keys (a NaN key lies beyond +/-inf);
//   * scale/zero point per group, computed redundantly by the 16 lanes of the row, with
//     the reference's per-op bf16 rounding (RNE after each op: v_cvt_pk_bf16_f32);
//   * per element: RN_bf16(x * RN_f32(1/s)) == RN_bf16(x / s) for every bf16 x and every
//     bf16 s >= RN_bf16(1e-10) (verified exhaustively: oracle/verify_recip.c), so one
//     v_pk_mul_f32 replaces the division; + z, RNE, round-half-even, clamp, pack;
//   * each lane emits exactly one packed int32 (4-bit) — 256 B contiguous per store;
//   * buffer descriptors are based at the tile start with the tile's byte length, so
//     slots past the tile end read zeros and their stores are dropped by the hardware
//     range check (no per-lane masks, no OOB access, tensors > 4 GB are fine).
// Ragged launches: one grid over the tiles of many tensors (descriptor table in HBM);
// waves grid-stride over tiles and advance a tensor cursor monotonically.
#include <cstdlib>

#include "awq_internal.h"

namespace awq {
namespace {

typedef short s2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __bf16 b2 __attribute__((ext_vector_type(2)));
typedef uint32_t u4 __attribute__((ext_vector_type(4)));
typedef uint32_t u2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes,
                                             0x00020000);
}

__device__ __forceinline__ s2 key2(uint32_t u) {
    s2 h = __builtin_bit_cast(s2, u);
    return h ^ ((h >> (s2)15) & (s2)0x7FFF);
}

__device__ __forceinline__ float key_to_f32(int key16) {
    // key16: sign-extended int16 key; the same involution maps it back to bf16 bits
    uint32_t h = (uint32_t)(key16 ^ ((key16 >> 15) & 0x7FFF)) & 0xFFFFu;
    return __uint_as_float(h << 16);
}

__device__ __forceinline__ f2 rn_bf16x2(f2 v) {
    b2 h = __builtin_convertvector(v, b2);
    return __builtin_convertvector(h, f2);
}

__device__ __forceinline__ float rn_bf16(float v) { return (float)(__bf16)v; }

template <int CTRL>
__device__ __forceinline__ s2 dpp_max(s2 w) {
    int o = __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, w), CTRL, 0xF, 0xF, false);
    return __builtin_elementwise_max(w, __builtin_bit_cast(s2, o));
}

struct GroupParams {
    float r;        // RN_f32(1 / s)
    float z;        // zero point (integral float; NaN possible only when special)
    float s;        // scale (bf16 value)
    bool special;   // s not finite: NaN/inf semantics needed per element
};

// awq.py:192-211 on one group, from the row-reduced keys.  QR = qmax - qmin.
template <int BITS, bool SYM>
__device__ __forceinline__ GroupParams group_params(s2 w) {
    constexpr float QR = (float)((1 << BITS) - 1);
    constexpr float INV_QR = 1.0f / QR;               // RN_f32(1/15), RN_f32(1/255)
    const float LO = __uint_as_float(0x2EDC0000u);    // RN_bf16(1e-10) = 1.0004442e-10
    int mxk = (int)w.x;
    int mnk = ~(int)w.y;
    bool nan = (mxk > 0x7F80) || (mnk < -32641);      // keys beyond +inf / -inf
    float mx = key_to_f32(mxk), mn = key_to_f32(mnk);
    if (nan) { mx = __builtin_nanf(""); mn = mx; }   // torch min/max both propagate NaN
    if (SYM) {                                        // awq.py:196-199
        float a = __builtin_fmaxf(__builtin_fabsf(mn), __builtin_fabsf(mx));
        if (nan) a = mx;
        mn = -a;
        mx = a;
    }
    float d = rn_bf16(mx - mn);                       // awq.py:202  bf16 subtract
    float s = rn_bf16(d * INV_QR);                    //             bf16 / (qmax-qmin)
    if (!__builtin_isnan(s)) s = __builtin_fmaxf(s, LO);   // awq.py:205 clamp(min=1e-10)
    GroupParams p;
    p.s = s;
    p.r = 1.0f / s;                                   // correctly rounded (no fast-math)
    if (SYM) {
        p.z = 0.0f;                                   // awq.py:208
    } else {
        float y = rn_bf16(mn * p.r);                  // == RN_bf16(mn / s)
        float z = __builtin_rintf(-y);                // awq.py:210-211 (qmin = 0)
        if (!__builtin_isnan(z)) z = __builtin_fminf(__builtin_fmaxf(z, 0.0f), QR);
        p.z = z;
    }
    p.special = !__builtin_isfinite(s);
    return p;
}

// Quantize the 8 bf16 of one lane (awq.py:245-248).  nib[i] = q_i - qmin.
template <int BITS, bool SYM>
__device__ __forceinline__ void quant8_fast(const u4 v, const GroupParams& p, uint32_t (&nib)[8]) {
    constexpr float QR = (float)((1 << BITS) - 1);
    constexpr float HALF = (float)(1 << (BITS - 1));
    const uint32_t src[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        f2 x = {__uint_as_float(src[i] << 16), __uint_as_float(src[i] & 0xFFFF0000u)};
        f2 t = rn_bf16x2(x * p.r);                   // RN_bf16(x / s)
        f2 u;
        if (SYM) {
            u = t + HALF;                             // rint(t)+8 == rint(t+8): exact shift
        } else {
            u = rn_bf16x2(t + p.z);                   // RN_bf16(x/s + z)
        }
        float u0 = __builtin_fminf(__builtin_fmaxf(__builtin_rintf(u.x), 0.0f), QR);
        float u1 = __builtin_fminf(__builtin_fmaxf(__builtin_rintf(u.y), 0.0f), QR);
        nib[2 * i] = (uint32_t)u0;
        nib[2 * i + 1] = (uint32_t)u1;
    }
}

// Same with the reference's NaN/inf semantics (groups whose scale is inf or NaN).
template <int BITS, bool SYM>
__device__ __forceinline__ void quant8_special(const u4 v, const GroupParams& p, uint32_t (&nib)[8],
                                            int32_t (&q)[8]) {
    constexpr int QMIN = SYM ? -(1 << (BITS - 1)) : 0;
    constexpr int QMAX = SYM ? (1 << (BITS - 1)) - 1 : (1 << BITS) - 1;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    const uint32_t src[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        uint32_t bits = (i & 1) ? (src[i >> 1] & 0xFFFF0000u) : (src[i >> 1] << 16);
        float x = __uint_as_float(bits);
        float t = rn_bf16(x * p.r);
        float u = SYM ? t : rn_bf16(t + p.z);
        float r = __builtin_rintf(u);
        int32_t qi;
        if (__builtin_isnan(r)) {
            qi = INT32_MIN;
        } else {
            r = __builtin_fminf(__builtin_fmaxf(r, (float)QMIN), (float)QMAX);
            qi = (int32_t)r;
        }
        q[i] = qi;
        nib[i] = ((uint32_t)qi - (uint32_t)QMIN) & MASK;
    }
}

__device__ __forceinline__ uint16_t f16_bits(float s) {
    if (__builtin_isnan(s)) return 0x7E00;
    _Float16 h = (_Float16)s;                          // v_cvt_f16_f32: RNE, subnormals kept
    return __builtin_bit_cast(uint16_t, h);
}

template <int BITS, bool SYM>
__device__ __forceinline__ void do_tile(const awq_tensor_desc& d, uint32_t tile, uint32_t* zw) {
    constexpr int QMIN = SYM ? -(1 << (BITS - 1)) : 0;
    const int lane = threadIdx.x & 63;
    const int row = lane >> 4;       // lane-row: 16 lanes = one group
    const int c = lane & 15;         // 16-B chunk of the group

    const TensorGeom g = fast_geom(d.rows, d.K, BITS);
    const uint32_t w0 = tile * g.WPT;
    const uint32_t w1 = min(w0 + g.WPT, g.words);
    const uint32_t start = word_group(g, w0);
    const uint32_t end = (w1 == g.words) ? (uint32_t)d.rows * g.G : word_group(g, w1);
    const uint32_t ng = end - start;            // groups in this tile (<= 16)

    const uint16_t* wp = (const uint16_t*)d.w + (uint64_t)start * kGroup;
    const __amdgpu_buffer_rsrc_t rw = rsrc(wp, ng * 256u);

    u4 v[4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)((4 * j + row) * 256 + c * 16), 0, 0);

    float sc[4];
    float zz[4];
    const bool want_tq = d.tensor_q != nullptr;
    const bool want_qz = d.qzeros != nullptr;
    if (want_qz && lane < 16) zw[lane] = 0u;

#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int slot = 4 * j + row;
        // ---- group min/max (awq.py:192-193) ----
        s2 k0 = key2(v[j].x), k1 = key2(v[j].y), k2 = key2(v[j].z), k3 = key2(v[j].w);
        s2 mx = __builtin_elementwise_max(__builtin_elementwise_max(k0, k1), __builtin_elementwise_max(k2, k3));
        s2 mn = __builtin_elementwise_min(__builtin_elementwise_min(k0, k1), __builtin_elementwise_min(k2, k3));
        s2 a = {mx.x, (short)~mn.x};
        s2 b = {mx.y, (short)~mn.y};
        s2 wv = __builtin_elementwise_max(a, b);
        wv = dpp_max<0xB1>(wv);    // quad_perm [1,0,3,2]
        wv = dpp_max<0x4E>(wv);    // quad_perm [2,3,0,1]
        wv = dpp_max<0x141>(wv);   // row_half_mirror
        wv = dpp_max<0x140>(wv);   // row_mirror: all 16 lanes hold the group's (max, ~min)
        const GroupParams p = group_params<BITS, SYM>(wv);
        sc[j] = p.s;
        zz[j] = p.z;

        uint32_t nib[8];
        int32_t q[8];
        if (__builtin_expect(p.special, 0)) {
            quant8_special<BITS, SYM>(v[j], p, nib, q);
        } else {
            quant8_fast<BITS, SYM>(v[j], p, nib);
#pragma unroll
            for (int i = 0; i < 8; ++i) q[i] = (int32_t)nib[i] + QMIN;
        }
        // ---- packed qweight: 4-bit -> one dword per lane, 8-bit -> two ----
        if (d.qweight) {
            if (BITS == 4) {
                uint32_t word = 0;
#pragma unroll
                for (int i = 0; i < 8; ++i) word |= nib[i] << (4 * i);
                __amdgpu_buffer_rsrc_t rq = rsrc(d.qweight + (uint64_t)start * 16, ng * 64u);
                __builtin_amdgcn_raw_buffer_store_b32(word, rq, (uint32_t)((slot * 16 + c) * 4), 0, 0);
            } else {
                u2v word;
                word.x = nib[0] | (nib[1] << 8) | (nib[2] << 16) | (nib[3] << 24);
                word.y = nib[4] | (nib[5] << 8) | (nib[6] << 16) | (nib[7] << 24);
                __amdgpu_buffer_rsrc_t rq = rsrc(d.qweight + (uint64_t)start * 32, ng * 128u);
                __builtin_amdgcn_raw_buffer_store_b64(word, rq, (uint32_t)((slot * 32 + 2 * c) * 4), 0, 0);
            }
        }
        // ---- reference-layout int32 tensor_q (parity mode) ----
        if (want_tq) {
            __amdgpu_buffer_rsrc_t rt = rsrc(d.tensor_q + (uint64_t)start * kGroup, ng * 512u);
            u4 lo = {(uint32_t)q[0], (uint32_t)q[1], (uint32_t)q[2], (uint32_t)q[3]};
            u4 hi = {(uint32_t)q[4], (uint32_t)q[5], (uint32_t)q[6], (uint32_t)q[7]};
            __builtin_amdgcn_raw_buffer_store_b128(lo, rt, (uint32_t)((slot * kGroup + 8 * c) * 4), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(hi, rt, (uint32_t)((slot * kGroup + 8 * c) * 4 + 16), 0, 0);
        }
        // ---- qzeros nibble into the tile's word (LDS, wave-private) ----
        if (want_qz && c == 0 && (uint32_t)slot < ng) {
            const uint32_t fg = start + (uint32_t)slot;
            uint32_t wi, pos;
            if (g.G % g.C == 0) {
                wi = fg / g.C;
                pos = fg % g.C;
            } else {
                uint32_t r = fg / g.G;
                uint32_t gg = fg - r * g.G;
                wi = r * g.WPR + gg / g.C;
                pos = gg % g.C;
            }
            uint32_t zn = __builtin_isnan(p.z) ? (uint32_t)(0u - (uint32_t)QMIN) : (uint32_t)((int)p.z - QMIN);
            zn &= (1u << BITS) - 1u;
            atomicOr(&zw[wi - w0], zn << (BITS * pos));
        }
    }
    // ---- per-group scalars: lane (c == j) of row `row` writes slot 4j+row (one store) ----
    {
        const int jj = c & 3;
        float s_sel = sc[0], z_sel = zz[0];
#pragma unroll
        for (int j = 1; j < 4; ++j) {
            if (jj == j) { s_sel = sc[j]; z_sel = zz[j]; }
        }
        const uint32_t slot = 4u * (uint32_t)jj + (uint32_t)row;
        if (c < 4) {
            if (d.scales) {
                __amdgpu_buffer_rsrc_t rs = rsrc(d.scales + start, ng * 2u);
                __builtin_amdgcn_raw_buffer_store_b16(f16_bits(s_sel), rs, slot * 2u, 0, 0);
            }
            if (d.zeros) {
                __amdgpu_buffer_rsrc_t rz = rsrc(d.zeros + start, ng * 4u);
                int32_t zi = __builtin_isnan(z_sel) ? INT32_MIN : (int32_t)z_sel;
                __builtin_amdgcn_raw_buffer_store_b32((uint32_t)zi, rz, slot * 4u, 0, 0);
            }
        }
    }
    if (want_qz) {
        const uint32_t nw = w1 - w0;
        if ((uint32_t)lane < nw) {
            __amdgpu_buffer_rsrc_t rz = rsrc(d.qzeros + w0, nw * 4u);
            __builtin_amdgcn_raw_buffer_store_b32(zw[lane], rz, (uint32_t)lane * 4u, 0, 0);
        }
    }
}

template <int BITS, bool SYM>
__global__ __launch_bounds__(256) void awq_fast_kernel(const awq_tensor_desc* __restrict__ descs,
                                                       awq_tensor_desc single, int n,
                                                       int64_t total_tiles) {
    __shared__ uint32_t zwords[kWavesPerBlock][kSlots];
    // wave index made provably uniform so tile/tensor bookkeeping and the buffer
    // descriptors live in SGPRs (no waterfall loops around the descriptors)
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t wave = (int64_t)blockIdx.x * kWavesPerBlock + wid;
    const int64_t nwaves = (int64_t)gridDim.x * kWavesPerBlock;
    int64_t t = wave;
    if (t >= total_tiles) return;
    if (descs == nullptr) {
        for (; t < total_tiles; t += nwaves) do_tile<BITS, SYM>(single, (uint32_t)t, zwords[wid]);
        return;
    }
    // first tensor of this wave: binary search on tile_begin (sorted, uniform)
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        int mid = (lo + hi + 1) >> 1;
        if (descs[mid].tile_begin <= t) lo = mid; else hi = mid - 1;
    }
    int cur = lo;
    awq_tensor_desc d = descs[cur];
    for (; t < total_tiles; t += nwaves) {
        bool moved = false;
        while (cur + 1 < n && descs[cur + 1].tile_begin <= t) { ++cur; moved = true; }
        if (moved) d = descs[cur];
        do_tile<BITS, SYM>(d, (uint32_t)(t - d.tile_begin), zwords[wid]);
    }
}

}  // namespace

hipError_t launch_fast(const awq_tensor_desc* descs_dev, const awq_tensor_desc* single, int n,
                       int64_t total_tiles, int bits, int symmetric, hipStream_t stream) {
    if (total_tiles <= 0) return hipSuccess;
    // grid: enough waves to keep ~8 x 16 KiB of loads in flight per CU, grid-stride beyond
    int64_t max_blocks = 256 * 8;
    if (const char* e = getenv("AWQ_HIP_MAX_BLOCKS")) {   // testing: force grid-stride loops
        long v = atol(e);
        if (v > 0) max_blocks = v;
    }
    int64_t blocks = (total_tiles + kWavesPerBlock - 1) / kWavesPerBlock;
    if (blocks > max_blocks) blocks = max_blocks;
    awq_tensor_desc one{};
    if (single) one = *single;
    dim3 grid((unsigned)blocks), block(256);
#define AWQ_LAUNCH(B, S) \
    hipLaunchKernelGGL((awq_fast_kernel<B, S>), grid, block, 0, stream, descs_dev, one, n, total_tiles)
    if (bits == 4 && !symmetric) AWQ_LAUNCH(4, false);
    else if (bits == 4) AWQ_LAUNCH(4, true);
    else if (!symmetric) AWQ_LAUNCH(8, false);
    else AWQ_LAUNCH(8, true);
#undef AWQ_LAUNCH
    return hipPeekAtLastError();
}

}  // namespace awq
