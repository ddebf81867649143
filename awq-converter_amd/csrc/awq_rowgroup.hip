// awq_rowgroup.hip — row-segment quantizer: bf16 / fp16 / fp32 weights with any group size
// up to 512 (fp32: 256) and any row length K (gfx950).
//
// Serves the reference's arbitrary group_size (src/awq_quantizer/quantization/awq.py:102,
// 286-374: groups along each row, the last zero-padded, awq.py:337-339) outside the
// streaming kernel's 32 / 64 / 128 / 256, with the same per-group arithmetic
// (awq.py:173-250; awq_quant.h) and packed outputs written directly.
#include "awq_quant.h"

namespace awq {
namespace {

// ---------------------------------------------------------------------------------------
// Any group size up to 512 (bf16 / fp16; 256 for fp32), any K: row-segment tiles.
//
// A tile = GPT consecutive groups of one row (GPT a multiple of 8 up to 64; the cost model
// picks 8, 16, 32 or 64), one 64-lane wave per tile:
//   stage   the segment's bytes go to LDS with 16-B loads, all in flight at once (16-B
//           aligned start; the tensor's last bytes go by 2-B loads);
//   pass 1  lane (grp, j) owns chunk j of group grp (P lanes per group = the largest power
//           of two <= 64 / the tile's groups, C = ceil(L / P) elements each) and reduces
//           the raw-bits min/max over it (packed 16-bit max/min, two chains) and over the
//           group's P lanes, then computes the group's parameters (the streaming kernel's
//           group_range / params_from_range: the same verified arithmetic) into LDS;
//   pass 2  lane = 8 consecutive elements (one qweight word at 4 bits): parameters from LDS
//           per half (L % 4 == 0) or per element, the field chain (bf16: packed f32 mul /
//           add), one coalesced word store.
// Tile boundaries fall on qweight and qzeros word boundaries (GPT * L and GPT are multiples
// of 8), so no word is shared between waves.  Replaces the one-wave-per-group generic
// kernel plus its int32 staging and pack passes (~10.5 B moved per element) for these
// shapes.
// ---------------------------------------------------------------------------------------
constexpr int kRgStageBytes = 8192;    // eligibility: 8 groups fit (any GPT the cost model picks)
constexpr int kRgStageMax = 16384;     // tuning override ceiling (rg_gpt)

template <typename F>
struct RgSlot {
    typedef typename std::conditional<F::kBytes == 2, uint16_t, uint32_t>::type T;
    static constexpr uint32_t kNan = F::kBytes == 2 ? 0xFFFFu : 0xFFFFFFFFu;   // field code of NaN
    __device__ static int sext(uint32_t v) { return F::kBytes == 2 ? (int)(int16_t)v : (int)v; }
    __device__ static float dec(uint32_t v) { return F::kBytes == 2 ? F::dec(v) : __uint_as_float(v); }
};

// packed field (q - qmin) of one element of a group with a positive finite scale, before
// the round + clamp (pack8_cvt / field_q)
template <typename F, int BITS, bool SYM, bool PLAIN>
__device__ __forceinline__ float field1_fast(float x, float r, float z, float s) {
    constexpr float HALF = (float)(1 << (BITS - 1));
    const float t = PLAIN ? F::quot_plain(x, r) : F::quot(x, s, r);
    float u;
    if (SYM && F::kWide) u = __builtin_rintf(t) + HALF;
    else if (SYM) u = t + HALF;
    else u = F::rn(t + F::as_fmt(z));
    return u;
}

// the field's value: clamp(rint(u), 0, 2^BITS - 1)
template <int BITS>
__device__ __forceinline__ float field_q(float u) {
    return __builtin_fminf(__builtin_fmaxf(__builtin_rintf(u), 0.0f), (float)((1 << BITS) - 1));
}

// the same for 8 bf16 elements, multiply and add as packed f32 pairs (v_pk_mul_f32 /
// v_pk_add_f32: each half is the IEEE f32 op, rounded to bf16 after it as above)
template <int BITS, bool SYM>
__device__ __forceinline__ void field8_bf16(const float (&x)[8], const float (&r)[8], const float (&z)[8],
                                            float (&q)[8]) {
    constexpr float HALF = (float)(1 << (BITS - 1));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f2 p = (f2){x[2 * i], x[2 * i + 1]} * (f2){r[2 * i], r[2 * i + 1]};
        const f2 t = {rn_bf16(p.x), rn_bf16(p.y)};
        f2 u;
        if (SYM) {
            u = t + (f2){HALF, HALF};                       // exact (as field1_fast)
        } else {
            const f2 a = t + (f2){z[2 * i], z[2 * i + 1]};
            u = (f2){rn_bf16(a.x), rn_bf16(a.y)};
        }
        q[2 * i] = u.x;
        q[2 * i + 1] = u.y;
    }
}

// raw-bits min/max over each aligned block of 2^lgP lanes (a group's lanes in pass 1):
// DPP quad / mirror steps and the row-pair swaps (wave-uniform lgP), every lane ends with
// its block's result
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ void rg_step(int& smax, uint32_t& umax, uint32_t& umin) {
    smax = max(smax, (int)dpp_mov<CTRL>((uint32_t)smax));
    umax = max(umax, dpp_mov<CTRL>(umax));
    umin = min(umin, dpp_mov<CTRL>(umin));
}
__device__ __forceinline__ void rg_reduce(int& smax, uint32_t& umax, uint32_t& umin, int lgP) {
    if (lgP >= 1) rg_step<0xB1>(smax, umax, umin);     // quad_perm [1,0,3,2]
    if (lgP >= 2) rg_step<0x4E>(smax, umax, umin);     // quad_perm [2,3,0,1]
    if (lgP >= 3) rg_step<0x141>(smax, umax, umin);    // row_half_mirror
    if (lgP >= 4) rg_step<0x140>(smax, umax, umin);    // row_mirror
    if (lgP >= 5) {                                    // rows 2k <-> 2k+1
        const auto a = __builtin_amdgcn_permlane16_swap((unsigned)smax, (unsigned)smax, false, false);
        const auto b = __builtin_amdgcn_permlane16_swap(umax, umax, false, false);
        const auto c = __builtin_amdgcn_permlane16_swap(umin, umin, false, false);
        smax = max((int)a[0], (int)a[1]);
        umax = max((uint32_t)b[0], (uint32_t)b[1]);
        umin = min((uint32_t)c[0], (uint32_t)c[1]);
    }
    if (lgP >= 6) {                                    // halves
        const auto a = __builtin_amdgcn_permlane32_swap((unsigned)smax, (unsigned)smax, false, false);
        const auto b = __builtin_amdgcn_permlane32_swap(umax, umax, false, false);
        const auto c = __builtin_amdgcn_permlane32_swap(umin, umin, false, false);
        smax = max((int)a[0], (int)a[1]);
        umax = max((uint32_t)b[0], (uint32_t)b[1]);
        umin = min((uint32_t)c[0], (uint32_t)c[1]);
    }
}

#define AWQ_RG_UNROLL 8

// raw-bits (signed max, unsigned max, unsigned min) of the 16-bit stage slots [s_lo, s_hi),
// s_hi > s_lo, from the identities: packed 16-bit max/min over whole dwords (two chains); an
// edge dword holding one foreign element gets a copy of its own element there
[[maybe_unused]] __device__ __forceinline__ void rg_range16(const uint32_t* st32, int s_lo, int s_hi, int& smax, uint32_t& umax,
                                           uint32_t& umin) {
    const int d_lo = s_lo >> 1, d_hi = (s_hi + 1) >> 1;
    s2 sm = {(short)-32768, (short)-32768}, sm_b = sm;
    us2 um = {0, 0}, um_b = um;
    us2 un = {(unsigned short)0xFFFF, (unsigned short)0xFFFF}, un_b = un;
    auto acc = [&](uint32_t v) {
        sm = __builtin_elementwise_max(sm, as_s2(v));
        um = __builtin_elementwise_max(um, as_us2(v));
        un = __builtin_elementwise_min(un, as_us2(v));
    };
    auto acc_b = [&](uint32_t v) {
        sm_b = __builtin_elementwise_max(sm_b, as_s2(v));
        um_b = __builtin_elementwise_max(um_b, as_us2(v));
        un_b = __builtin_elementwise_min(un_b, as_us2(v));
    };
    uint32_t first = st32[d_lo];
    if (s_lo & 1) first = __builtin_amdgcn_perm(first, first, 0x03020302u);   // low half := high
    if (d_hi - d_lo == 1 && (s_hi & 1)) first = __builtin_amdgcn_perm(first, first, 0x01000100u);
    acc(first);
    if (d_hi - d_lo > 1) {
        int d = d_lo + 1;
        for (; d + 4 <= d_hi - 1; d += 4) {
            const uint32_t v0 = st32[d], v1 = st32[d + 1], v2 = st32[d + 2], v3 = st32[d + 3];
            acc(v0);
            acc_b(v1);
            acc(v2);
            acc_b(v3);
        }
        if (d + 2 <= d_hi - 1) {
            const uint32_t v0 = st32[d], v1 = st32[d + 1];
            acc(v0);
            acc_b(v1);
            d += 2;
        }
        if (d < d_hi - 1) acc_b(st32[d]);
        uint32_t last = st32[d_hi - 1];
        if (s_hi & 1) last = __builtin_amdgcn_perm(last, last, 0x01000100u);        // high half := low
        acc(last);
    }
    sm = __builtin_elementwise_max(sm, sm_b);
    um = __builtin_elementwise_max(um, um_b);
    un = __builtin_elementwise_min(un, un_b);
    smax = max((int)sm.x, (int)sm.y);
    umax = (uint32_t)max((int)um.x, (int)um.y);
    umin = (uint32_t)min((int)un.x, (int)un.y);
}

// LDS: the segment's stage (dynamic, sized by the launch to the tile: 1.6-8 KiB) + 1.3 KiB
template <typename F, int BITS, bool SYM, int SPLIT, bool P1C, bool TQ>
__global__ __launch_bounds__(128) void awq_rowgroup_kernel(const void* __restrict__ w, int64_t rows, int64_t K,
                                                             int64_t L, int lgP, int GPT, uint32_t tiles_per_row,
                                                             int64_t G, int C, float invL,
                                                             int32_t* __restrict__ qweight, int32_t* __restrict__ qzeros,
                                                             uint16_t* __restrict__ scales,
                                                             int32_t* __restrict__ tensor_q, int32_t* __restrict__ zeros,
                                                             uint32_t nan_code, int lgP_last, int C_last, int p2reg,
                                                             int ldsdma, int p1u) {
    typedef RgSlot<F> SL;
    typedef typename SL::T S;
#ifndef AWQ_DIAG
    ldsdma = 1;                            // the shipped library: LDS-DMA stage, no A/B switches
    p2reg = 0;
#endif
    constexpr int QMIN = SYM ? -(1 << (BITS - 1)) : 0;
    constexpr uint32_t MASK = (1u << BITS) - 1u;
    constexpr int PER = 32 / BITS;             // elements (and groups) per packed word
    constexpr uint32_t NANF = (uint32_t)(0u - (uint32_t)QMIN) & MASK;   // field of INT32_MIN - qmin
    extern __shared__ __attribute__((aligned(16))) unsigned char rg_lds[];
    S* stage = (S*)rg_lds;                              // rg_stage_bytes(): the segment + its alignment skew
    __shared__ __attribute__((aligned(16))) uint32_t zst[64];
    __shared__ float4 prm[64];                          // per group: r, z, s, special
    __shared__ int not_plain;                           // a group of the tile needs the full quotient
    __shared__ int any_special;                         // a group of the tile has scale 0 / inf / NaN
    __shared__ int acc_smax[P1C ? 64 : 1];              // P1C: per-group raw-bits reductions
    __shared__ uint32_t acc_umax[P1C ? 64 : 1], acc_umin[P1C ? 64 : 1];
    // one tile per workgroup of 1 or 2 waves (host-chosen: two waves share a large tile's LDS
    // stage, so a whole-row tile keeps 8 waves per SIMD resident)
    const int lane = threadIdx.x, NT = blockDim.x;
    // (host-side G, C, log2 P and a 32-bit tile split: 64-bit divisions per wave on the
    //  CU's shared scalar unit were a visible part of the per-tile cost)
    const uint32_t tile = blockIdx.x;   // (an XCD-contiguous tile order measured no different: r2z3)
    // (whole-row tiles, the common case, need no division: the scalar unit has no divider)
    const uint32_t r32 = tiles_per_row == 1 ? tile : tile / tiles_per_row;
    const int64_t r = r32;
    // (32-bit row geometry: the host admits rows of < 2^30 elements; the scalar unit has no
    //  64-bit compare, so 64-bit min()s went through VALU compares)
    const int K32 = (int)K, L32g = (int)L;
    const int g0 = (int)(tile - r32 * tiles_per_row) * GPT;
    const int ng = min(GPT, (int)G - g0);
    if (ng < GPT) {   // the row's last, partial tile: more lanes per group (host-computed)
        lgP = lgP_last;
        C = C_last;
    }
    const int P = 1 << lgP;
    const int kb = g0 * L32g;                                    // the row segment [kb, kb + n_el)
    const int n_el = min((g0 + ng) * L32g, K32) - kb;
    // ---- stage the segment's bytes (from a 16-B aligned start) in LDS ----
    const uint64_t byte0 = ((uint64_t)r32 * (uint64_t)K32 + (uint64_t)kb) * F::kBytes;
    const uint64_t a0 = byte0 & ~(uint64_t)15;
    const int skew = (int)(byte0 - a0) / F::kBytes;               // slot of element kb
    const uint64_t total = (uint64_t)rows * (uint64_t)K * F::kBytes;
    const int nbytes = (int)(byte0 - a0) + n_el * F::kBytes;
    const int nch = (nbytes + 15) >> 4;
    const uint64_t rem = total - a0;                              // bytes from a0 to the tensor end
    const uint32_t lim = (rem >> 32) ? 16u * (uint32_t)nch : min((uint32_t)rem, 16u * (uint32_t)nch);
    const __amdgpu_buffer_rsrc_t rw = rsrc((const char*)w + a0, lim);
    u4 vreg[4];                              // the 4-chunk stage's loads, reused by pass 2
    if (__builtin_expect(16u * (uint32_t)nch <= lim, 1) && ldsdma) {
        // every 16-B chunk of the segment straight from memory into its stage slot (LDS-DMA:
        // no VGPR round trip, no LDS store instructions, every load in flight before one
        // wait).  Lane t of wave w writes slot base + 16 t, so a wave's loads go to its own
        // 64-chunk window of each NT-chunk step.
        const int wbase = __builtin_amdgcn_readfirstlane(lane & ~63);
        if (nch == 4 * NT) {
            // exactly 4 chunks per lane (a 4 096-element 16-bit row on two waves): four
            // unmasked global DMAs, unrolled (round 4, r4c: -2..5 % against the register stage
            // with pass 2 from registers; r4d: the masked buffer loop below lost 2..5 % here)
            const char* src = (const char*)w + a0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                __builtin_amdgcn_global_load_lds((const void*)(src + 16 * (NT * k + lane)),
                                                 (__attribute__((address_space(3))) void*)((char*)stage +
                                                                                          16 * (NT * k + wbase)),
                                                 16, 0, 0);
        } else {
            // any other segment: range-checked buffer DMAs, lanes past the segment masked off
            // (r4d: -5..7 % at K = 3000, -1..2 % at K = 14336 against the register stage)
#pragma unroll 4
            for (int c0 = 0; c0 < nch; c0 += NT) {
                if (c0 + lane < nch)
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        rw, (__attribute__((address_space(3))) void*)((char*)stage + 16 * (c0 + wbase)), 16,
                        (uint32_t)(16 * (c0 + lane)), 0, 0, AWQ_LOAD_AUX);
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (__builtin_expect(16u * (uint32_t)nch <= lim, 1)) {
        // (diagnostics A/B, rg_ldsdma = 1: the round-3 register stage)
        // every 16-B load of the segment in flight before the first LDS store (a load ->
        // store loop waits out one memory round trip per load).  All 8 loads are issued
        // unconditionally: offsets past the segment fall outside the buffer range (lim) and
        // read zeros without a memory access, and no register needs a value on a skipped
        // path (conditional loads cost 28 v_mov per wave of phi copies); lanes past the end
        // store nothing
        if (nch == 4 * NT) {
            // (exactly 4 chunks per lane — a 4 096-element bf16 row on two waves: 4 loads
            //  and 4 unmasked stores, no range-checked dummy loads; the chunks stay in
            //  registers for pass 2, whose lane -> chunk map is the same)
#pragma unroll
            for (int k = 0; k < 4; ++k)
                vreg[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)(16 * (NT * k + lane)), 0, AWQ_LOAD_AUX);
#pragma unroll
            for (int k = 0; k < 4; ++k) *(u4*)((char*)stage + 16 * (NT * k + lane)) = vreg[k];
        } else
        for (int c0 = 0; c0 < nch; c0 += 8 * NT) {
            u4 v[8];
#pragma unroll
            for (int k = 0; k < 8; ++k)
                v[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)(16 * (c0 + NT * k + lane)), 0, AWQ_LOAD_AUX);
#pragma unroll
            for (int k = 0; k < 8; ++k)
                if (c0 + NT * k + lane < nch) *(u4*)((char*)stage + 16 * (c0 + NT * k + lane)) = v[k];
        }
    } else
#pragma unroll 4
    for (int c = lane; c < nch; c += NT) {
        if (__builtin_expect(16u * c + 16u <= lim, 1)) {
            *(u4*)((char*)stage + 16 * c) = __builtin_amdgcn_raw_buffer_load_b128(rw, (uint32_t)(16 * c), 0, AWQ_LOAD_AUX);
        } else {   // the tensor's last bytes: a 16-B load straddling the range end would read as all zeros
            for (int h = 0; h < 8; ++h)
                ((uint16_t*)stage)[8 * c + h] = __builtin_amdgcn_raw_buffer_load_b16(rw, (uint32_t)(16 * c + 2 * h), 0, 0);
        }
    }
    if (lane == 0) {
        not_plain = 0;
        any_special = 0;
    }
    // uniform pass 1 (host: 16-bit, even K and L, P | L with an even L / P for every tile):
    // the row's zero-padded last group gets its padding as real zeros in the stage
    // (awq.py:337-339), so every lane reduces exactly C elements with no bounds.  Past a
    // segment that ends inside a 16-B chunk the slots hold the chunk's foreign bytes, which
    // another wave may have staged: there the zeros go in after a barrier.
    const int pad = (F::kBytes == 2 && p1u) ? ng * L32g - n_el : 0;
    const bool pad_late = pad > 0 && ((skew + n_el) & 7) != 0;
    if (pad > 0 && !pad_late)
        for (int i = lane; i < pad; i += NT) ((uint16_t*)stage)[skew + n_el + i] = 0;
    // TQ: the parity outputs (tensor_q) are wanted (a compile-time switch: the packed-only
    // kernel carries no per-sweep checks for them)
    if constexpr (!TQ) tensor_q = nullptr;
    if constexpr (P1C) {
        // identities; the row's zero-padded last group starts from 0 (awq.py:337-339: the
        // zeros join its min/max)
        if (lane < ng) {
            const bool pad = lane == ng - 1 && n_el - lane * (int)L < (int)L;
            acc_smax[lane] = pad ? 0 : INT_MIN;
            acc_umax[lane] = 0u;
            acc_umin[lane] = pad ? 0u : F::kOnes;
        }
    }
    __syncthreads();
    if (pad_late) {
        for (int i = lane; i < pad; i += NT) ((uint16_t*)stage)[skew + n_el + i] = 0;
        __syncthreads();
    }
    if constexpr (P1C) {
        // ---- pass 1, lanes split evenly over the tile's groups: Q = NT / ng lanes per group
        //      (any count — not only a power of two; 3 for 41 groups of a 128-lane tile where
        //      the by-groups pass keeps 2), each lane reduces one even-length run of its group
        //      and merges it into the group's LDS slots (ds_max / ds_min) ----
        const int Q = NT / ng;                            // >= 1: ng <= 64 <= NT
        const int grp = (int)((float)lane * __builtin_amdgcn_rcpf((float)Q) + 1e-3f);   // lane / Q (lane < 128)
        const int jq = lane - grp * Q;
        if (grp < ng) {
            const int glen = min((int)L, n_el - grp * (int)L);
            const int cq = ((glen + Q - 1) / Q + 1) & ~1;   // even: runs start on dword pairs
            const int cb = min(jq * cq, glen), ce = min(cb + cq, glen);
            if (ce > cb) {
                const int base = skew + grp * (int)L;
                int smx;
                uint32_t umx, umn;
                if constexpr (F::kBytes == 2) {
                    rg_range16((const uint32_t*)stage, base + cb, base + ce, smx, umx, umn);
                } else {
                    smx = INT_MIN;
                    umx = 0u;
                    umn = F::kOnes;
                    int i1 = cb;
                    for (; i1 + AWQ_RG_UNROLL <= ce; i1 += AWQ_RG_UNROLL) {
                        uint32_t v[AWQ_RG_UNROLL];
#pragma unroll
                        for (int u = 0; u < AWQ_RG_UNROLL; ++u) v[u] = stage[base + i1 + u];
#pragma unroll
                        for (int u = 0; u < AWQ_RG_UNROLL; ++u) {
                            smx = max(smx, SL::sext(v[u]));
                            umx = max(umx, v[u]);
                            umn = min(umn, v[u]);
                        }
                    }
                    for (; i1 < ce; ++i1) {
                        const uint32_t v = stage[base + i1];
                        smx = max(smx, SL::sext(v));
                        umx = max(umx, v);
                        umn = min(umn, v);
                    }
                }
                atomicMax(&acc_smax[grp], smx);
                atomicMax(&acc_umax[grp], umx);
                atomicMin(&acc_umin[grp], umn);
            }
        }
        __syncthreads();
        // ---- the tile's group parameters: one lane per group (wave 0: ng <= 64) ----
        if (lane < ng) {
            float gmn, gmx;
            bool gnan;
            group_range<F, SYM>(acc_smax[lane], acc_umax[lane], acc_umin[lane], gmn, gmx, gnan);
            const GroupParams p = params_from_range<F, BITS, SYM>(gmn, gmx);
            const bool special = !F::fast(p.r);
            if (F::kHasPlain && !F::plain_ok(p.s)) not_plain = 1;
            if (special) any_special = 1;
            const int64_t gi = r * G + g0 + lane;
            if (scales) scales[gi] = f16_bits(p.s, gnan, nan_code);
            if (zeros) zeros[gi] = __builtin_isnan(p.z) ? INT32_MIN : (int32_t)p.z;
            zst[lane] = __builtin_isnan(p.z) ? NANF : ((uint32_t)((int)p.z - QMIN) & MASK);
            prm[lane] = (float4){p.r, p.z, p.s, special ? 1.0f : 0.0f};
        }
    } else {
    // ---- this lane's chunk of its group ----
    const int grp = lane >> lgP, j = lane & (P - 1);
    const bool active = grp < ng;
    int smax;
    uint32_t umax, umin;
    if (F::kBytes == 2 && p1u) {
        // uniform: C (even) elements from a dword boundary for every lane — lanes past the
        // tile's groups re-read the last group (their results are not used) — in a loop whose
        // trip count is the same for the whole wave
        const uint32_t* p = (const uint32_t*)stage + ((skew + min(grp, ng - 1) * L32g + j * C) >> 1);
        const int nd = C >> 1;
        s2 sm = {(short)-32768, (short)-32768}, sm_b = sm;
        us2 um = {0, 0}, um_b = um;
        us2 un = {(unsigned short)0xFFFF, (unsigned short)0xFFFF}, un_b = un;
        int d = 0;
        for (; d + 4 <= nd; d += 4) {
            const uint32_t v0 = p[d], v1 = p[d + 1], v2 = p[d + 2], v3 = p[d + 3];
            sm = __builtin_elementwise_max(sm, as_s2(v0));
            um = __builtin_elementwise_max(um, as_us2(v0));
            un = __builtin_elementwise_min(un, as_us2(v0));
            sm_b = __builtin_elementwise_max(sm_b, as_s2(v1));
            um_b = __builtin_elementwise_max(um_b, as_us2(v1));
            un_b = __builtin_elementwise_min(un_b, as_us2(v1));
            sm = __builtin_elementwise_max(sm, as_s2(v2));
            um = __builtin_elementwise_max(um, as_us2(v2));
            un = __builtin_elementwise_min(un, as_us2(v2));
            sm_b = __builtin_elementwise_max(sm_b, as_s2(v3));
            um_b = __builtin_elementwise_max(um_b, as_us2(v3));
            un_b = __builtin_elementwise_min(un_b, as_us2(v3));
        }
        for (; d < nd; ++d) {
            const uint32_t v = p[d];
            sm = __builtin_elementwise_max(sm, as_s2(v));
            um = __builtin_elementwise_max(um, as_us2(v));
            un = __builtin_elementwise_min(un, as_us2(v));
        }
        sm = __builtin_elementwise_max(sm, sm_b);
        um = __builtin_elementwise_max(um, um_b);
        un = __builtin_elementwise_min(un, un_b);
        smax = max((int)sm.x, (int)sm.y);
        umax = (uint32_t)max((int)um.x, (int)um.y);
        umin = (uint32_t)min((int)un.x, (int)un.y);
    } else {
    const int glen = active ? min((int)L, n_el - grp * (int)L) : 0;   // elements in the row (tail: fewer)
    const int cb = min(j * C, glen), ce = min(cb + C, glen);
    const int base = skew + grp * (int)L;
    const bool padded = active && glen < L;                    // awq.py:337-339: zeros join the min/max
    smax = padded ? 0 : INT_MIN;
    umax = 0;
    umin = padded ? 0u : F::kOnes;
    if constexpr (F::kBytes == 2) {
        // raw 16-bit pairs with packed max/min (v_pk_*_i16/u16: two elements per instruction);
        // an edge dword holding one foreign element gets a copy of its own element there
        const int s_lo = base + cb, s_hi = base + ce;
        if (s_hi > s_lo) {
            const uint32_t* st32 = (const uint32_t*)stage;
            const int d_lo = s_lo >> 1, d_hi = (s_hi + 1) >> 1;
            s2 sm = {(short)(padded ? 0 : -32768), (short)(padded ? 0 : -32768)};
            us2 um = {0, 0};
            us2 un = {(unsigned short)(padded ? 0 : 0xFFFF), (unsigned short)(padded ? 0 : 0xFFFF)};
            s2 sm_b = sm;                                 // a second, independent set of chains
            us2 um_b = um, un_b = un;
            auto acc = [&](uint32_t v) {
                sm = __builtin_elementwise_max(sm, as_s2(v));
                um = __builtin_elementwise_max(um, as_us2(v));
                un = __builtin_elementwise_min(un, as_us2(v));
            };
            auto acc_b = [&](uint32_t v) {
                sm_b = __builtin_elementwise_max(sm_b, as_s2(v));
                um_b = __builtin_elementwise_max(um_b, as_us2(v));
                un_b = __builtin_elementwise_min(un_b, as_us2(v));
            };
            uint32_t first = st32[d_lo];
            if (s_lo & 1) first = __builtin_amdgcn_perm(first, first, 0x03020302u);   // low half := high
            if (d_hi - d_lo == 1 && (s_hi & 1)) first = __builtin_amdgcn_perm(first, first, 0x01000100u);
            acc(first);
            if (d_hi - d_lo > 1) {
                int d = d_lo + 1;
                for (; d + 4 <= d_hi - 1; d += 4) {
                    const uint32_t v0 = st32[d], v1 = st32[d + 1], v2 = st32[d + 2], v3 = st32[d + 3];
                    acc(v0);
                    acc_b(v1);
                    acc(v2);
                    acc_b(v3);
                }
                if (d + 2 <= d_hi - 1) {                  // <= 3 left: no loop
                    const uint32_t v0 = st32[d], v1 = st32[d + 1];
                    acc(v0);
                    acc_b(v1);
                    d += 2;
                }
                if (d < d_hi - 1) acc_b(st32[d]);
                uint32_t last = st32[d_hi - 1];
                if (s_hi & 1) last = __builtin_amdgcn_perm(last, last, 0x01000100u);        // high half := low
                acc(last);
            }
            sm = __builtin_elementwise_max(sm, sm_b);
            um = __builtin_elementwise_max(um, um_b);
            un = __builtin_elementwise_min(un, un_b);
            smax = max((int)sm.x, (int)sm.y);
            umax = (uint32_t)max((int)um.x, (int)um.y);
            umin = (uint32_t)min((int)un.x, (int)un.y);
        }
    } else {
        int i1 = cb;
        for (; i1 + AWQ_RG_UNROLL <= ce; i1 += AWQ_RG_UNROLL) {   // independent LDS reads in flight
            uint32_t v[AWQ_RG_UNROLL];
#pragma unroll
            for (int u = 0; u < AWQ_RG_UNROLL; ++u) v[u] = stage[base + i1 + u];
#pragma unroll
            for (int u = 0; u < AWQ_RG_UNROLL; ++u) {
                smax = max(smax, SL::sext(v[u]));
                umax = max(umax, v[u]);
                umin = min(umin, v[u]);
            }
        }
        for (; i1 < ce; ++i1) {
            const uint32_t v = stage[base + i1];
            smax = max(smax, SL::sext(v));
            umax = max(umax, v);
            umin = min(umin, v);
        }
    }
    }   // (per-lane bounds form)
    rg_reduce(smax, umax, umin, lgP);                          // the group's P lanes (aligned)
    float gmn, gmx;
    bool gnan;
    group_range<F, SYM>(smax, umax, umin, gmn, gmx, gnan);
    const GroupParams p = params_from_range<F, BITS, SYM>(gmn, gmx);
    const bool special = !F::fast(p.r);
    // wave-uniform: every group of the tile admits the plain quotient (F::plain_ok)
    if (F::kHasPlain && active && j == 0 && !F::plain_ok(p.s)) not_plain = 1;
    if (active && j == 0 && special) any_special = 1;
    if (active && j == 0) {
        const int64_t gi = r * G + g0 + grp;
        if (scales) scales[gi] = f16_bits(p.s, gnan, nan_code);
        if (zeros) zeros[gi] = __builtin_isnan(p.z) ? INT32_MIN : (int32_t)p.z;
        zst[grp] = __builtin_isnan(p.z) ? NANF : ((uint32_t)((int)p.z - QMIN) & MASK);
        prm[grp] = (float4){p.r, p.z, p.s, special ? 1.0f : 0.0f};
    }
    }   // (pass 1 by groups)
    __syncthreads();
    // uniform: every group of the tile admits the plain quotient (F::plain_ok)
    const bool plain = F::kHasPlain && not_plain == 0;
    // uniform: no group of the tile takes the IEEE-division path (skips the per-sweep checks)
    const bool tile_special = any_special != 0;
    // ---- pass 2: lane = 8 consecutive elements of the segment (one qweight word at 4 bits):
    //      its groups' parameters from LDS, quantize, pack, store (kb is a word boundary) ----
    const int nck = (n_el + 7) >> 3;
    const int L32 = (int)L;                               // invL = RN(1 / L): exact group index e * invL
                                                          // for e < 2^13, L <= 512 (host-computed)
    const int64_t wpr = (K + PER - 1) / PER;
    int32_t* qdst = qweight ? qweight + r * wpr + kb / PER : nullptr;
    // one chunk: c = its index in the segment, efA = 8 c + 0.5 (exact float); ALIGNED: the
    // segment starts 16-B aligned (skew 0); FULL: the chunk holds 8 elements of the row
    auto sweep = [&](int c, float efA, auto aligned_t, auto full_t, auto plain_t, auto special_t,
                     const u4* rv = nullptr) {
        constexpr bool ALIGNED = decltype(aligned_t)::value, FULL = decltype(full_t)::value;
        constexpr bool PLAIN = decltype(plain_t)::value;
        constexpr bool SPECIAL = decltype(special_t)::value;   // the tile has a special group
        const int e0c = 8 * c;
        const bool tail = !FULL && e0c + 8 > n_el;        // the row's last, partial chunk
        float x[8];
        u4 vraw = {0u, 0u, 0u, 0u};                       // (fp16 packed chain: the raw pairs)
        if constexpr (ALIGNED) {                          // 16-B aligned chunk (K % 8 == 0 rows)
            // (from the stage's registers when given; past n_el: the stage's slack)
            const u4 v0 = (F::kBytes == 2 && rv) ? *rv : *(const u4*)(stage + e0c);
            vraw = v0;
            if constexpr (F::kBytes == 2) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const uint32_t wd = v0[i];
                    x[2 * i] = F::lo(wd);
                    x[2 * i + 1] = F::hi(wd);
                }
            } else {
                const u4 v1 = *(const u4*)(stage + e0c + 4);
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    x[i] = __uint_as_float(v0[i]);
                    x[4 + i] = __uint_as_float(v1[i]);
                }
            }
        } else {
#pragma unroll
            for (int i = 0; i < 8; ++i) x[i] = SL::dec(stage[skew + min(e0c + i, n_el - 1)]);
        }
        // parameters per element.  SPLIT 8 (L % 8 == 0): the chunk lies in one group; SPLIT 4
        // (L % 4 == 0): each half does (no per-element selects); SPLIT 1: at most two groups
        // meet in the chunk when L >= 8, one lookup per element below that
        float rr[8], zz[8], ss[8];
        bool spec;
        if constexpr (SPLIT == 8 || SPLIT == 4) {
            const int gA = (int)(efA * invL);             // < ng: e0c < n_el
            const float4 pA = prm[gA];
            float4 pB = pA;
            if constexpr (SPLIT == 4) pB = prm[min((int)((efA + 4.0f) * invL), ng - 1)];
            spec = SPECIAL && (pA.w != 0.0f || pB.w != 0.0f);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                rr[i] = i < 4 ? pA.x : pB.x;
                zz[i] = i < 4 ? pA.y : pB.y;
                ss[i] = i < 4 ? pA.z : pB.z;
            }
        } else if (L32 >= 8) {
            const int gA = (int)(((float)e0c + 0.5f) * invL);
            const int bnd = (gA + 1) * L32 - e0c;         // first element of the next group
            const float4 pA = prm[gA], pB = prm[min(gA + 1, ng - 1)];
            spec = SPECIAL && (pA.w != 0.0f || (bnd < 8 && pB.w != 0.0f));
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const bool a = i < bnd;
                rr[i] = a ? pA.x : pB.x;
                zz[i] = a ? pA.y : pB.y;
                ss[i] = a ? pA.z : pB.z;
            }
        } else {
            spec = false;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int gi = min((int)(((float)(e0c + i) + 0.5f) * invL), ng - 1);
                const float4 pi = prm[gi];
                spec |= SPECIAL && pi.w != 0.0f;
                rr[i] = pi.x;
                zz[i] = pi.y;
                ss[i] = pi.z;
            }
        }
        int32_t qv[8];                                    // q (reference value), INT32_MIN for NaN
        uint32_t word0 = 0, word1 = 0;
        if constexpr (std::is_same<F, FmtF16>::value && PLAIN && ALIGNED && !TQ) {
            if (__builtin_expect(!spec && !tail, 1)) {    // fp16: the packed-pair chain
                const uint32_t d[4] = {vraw.x, vraw.y, vraw.z, vraw.w};
                pack8_f16_plain<BITS, SYM>(d, rr, zz, word0, word1);
                goto store;
            }
        }
        if (__builtin_expect(!spec, 1)) {
            float q[8];
            if constexpr (std::is_same<F, FmtBF16>::value) {
                field8_bf16<BITS, SYM>(x, rr, zz, q);
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    q[i] = field1_fast<F, BITS, SYM, PLAIN>(x[i], rr[i], zz[i], ss[i]);
            }
            if (__builtin_expect(tail, 0)) {
                const int nv = n_el - e0c;
#pragma unroll
                for (int i = 1; i < 8; ++i)
                    if (i >= nv) q[i] = 0.0f;             // past the row end: zero fields
            }
            if (tensor_q) {
#pragma unroll
                for (int i = 0; i < 8; ++i) qv[i] = (int32_t)field_q<BITS>(q[i]) + QMIN;
            }
            pack8_cvt<BITS>(q, word0, word1);
        } else {                                          // a group with scale 0 / inf / NaN: IEEE division
            constexpr int QMAX = SYM ? (1 << (BITS - 1)) - 1 : (1 << BITS) - 1;
            const int nv = n_el - e0c;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const float t = F::rn(opaque(x[i]) / ss[i]);
                const float u = SYM ? t : F::rn(t + zz[i]);
                const float rq = __builtin_rintf(u);
                int32_t qi = __builtin_isnan(rq) ? INT32_MIN
                                                 : (int32_t)__builtin_fminf(__builtin_fmaxf(rq, (float)QMIN), (float)QMAX);
                uint32_t f = ((uint32_t)qi - (uint32_t)QMIN) & MASK;
                if (i >= nv) { f = 0; qi = QMIN; }
                qv[i] = qi;
                if (BITS == 4) word0 |= f << (4 * i);
                else if (i < 4) word0 |= f << (8 * i);
                else word1 |= f << (8 * (i - 4));
            }
        }
    store:
        if (TQ ? qdst != nullptr : true) {            // (packed-only: pass 2 runs only with qweight)
            if (BITS == 4) {
                qdst[(uint32_t)c] = (int32_t)word0;            // (unsigned: a 32-bit offset on an SGPR base)
            } else {
                qdst[2u * (uint32_t)c] = (int32_t)word0;
                if (!tail || e0c + 4 < n_el) qdst[2u * (uint32_t)c + 1u] = (int32_t)word1;
            }
        }
        if (tensor_q) {
            int32_t* tq = tensor_q + r * K + kb + e0c;
            if (__builtin_expect(!tail, 1)) {
#pragma unroll
                for (int i = 0; i < 8; ++i) tq[i] = qv[i];
            } else {
                const int nv = n_el - e0c;
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    if (i < nv) tq[i] = qv[i];
            }
        }
    };
    // sweeps over the segment's chunks, lane = chunk c, c + NT, ...: the sweeps in which every
    // lane has a full chunk run as a uniform (scalar) loop with no per-lane bounds or tail
    // checks, the rest (<= 1 sweep of full chunks + the row's last partial chunk) guarded
    const float efStep = 8.0f * (float)NT;
    const int lgNT = NT == 128 ? 7 : 6;
    auto sweeps = [&](auto aligned_t, auto plain_t, auto special_t) {
        if constexpr (F::kBytes == 2 && decltype(aligned_t)::value) {
            if (p2reg && nch == 4 * NT && n_el == 32 * NT) {   // the 4-chunk stage: data in registers
                float efA = 8.0f * (float)lane + 0.5f;
#pragma unroll
                for (int sw = 0; sw < 4; ++sw, efA += efStep)
                    sweep(lane + (sw << lgNT), efA, aligned_t, std::true_type{}, plain_t, special_t, &vreg[sw]);
                return;
            }
        }
        const int full_sweeps = (n_el >> 3) >> lgNT;
        float efA = 8.0f * (float)lane + 0.5f;
        for (int sw = 0; sw < full_sweeps; ++sw, efA += efStep)
            sweep(lane + (sw << lgNT), efA, aligned_t, std::true_type{}, plain_t, special_t);
        for (int c = lane + (full_sweeps << lgNT); c < nck; c += NT, efA += efStep)
            sweep(c, efA, aligned_t, std::false_type{}, plain_t, special_t);
    };
    // (uniform switches hoisted out of the sweeps: the alignment and, for fp16, whether every
    //  group of the tile admits the plain quotient)
    // (and whether a group of the tile takes the IEEE-division path: without one the sweeps
    //  carry no per-lane special-value test, round 4)
    auto by_special = [&](auto aligned_t, auto plain_t) {
        if (tile_special) sweeps(aligned_t, plain_t, std::true_type{});
        else sweeps(aligned_t, plain_t, std::false_type{});
    };
    auto by_plain = [&](auto aligned_t) {
        if constexpr (F::kHasPlain) {
            if (plain) by_special(aligned_t, std::true_type{});
            else by_special(aligned_t, std::false_type{});
        } else {
            by_special(aligned_t, std::false_type{});
        }
    };
    // (the packed-only kernel's pass 2 exists for qweight: without it, none)
    if (TQ || qdst) {
        if (skew == 0) by_plain(std::true_type{});
        else by_plain(std::false_type{});
    }
    if (qzeros) {                                 // g0 is a word boundary: GPT % PER == 0
        const int64_t zpr = (G + PER - 1) / PER;
        const int nwz = (ng + PER - 1) / PER;
        if (lane < nwz) {                         // the word's PER fields: 16-B LDS reads, the
            const int nz = min(PER, ng - lane * PER); // slots past the tile's groups masked
            uint32_t zf[PER];
#pragma unroll
            for (int h = 0; h < PER / 4; ++h) {
                const u4 q4 = *(const u4*)&zst[lane * PER + 4 * h];
#pragma unroll
                for (int i = 0; i < 4; ++i) zf[4 * h + i] = q4[i];
            }
            uint32_t word = 0;
#pragma unroll
            for (int i = 0; i < PER; ++i) word |= (i < nz ? zf[i] : 0u) << (BITS * i);
            qzeros[r * zpr + g0 / PER + lane] = (int32_t)word;
        }
    }
}

}  // namespace

// Row-segment tiles of awq_rowgroup_kernel.  Whole-row tiles shared by two waves when a
// 16-bit row of >= 2560 elements has <= 64 groups and fits a 16 KiB stage (r2ae / r2af: a
// whole-row tile runs 1 059 VALU per row against 1 551 for 16-group one-wave tiles, and two
// waves per LDS stage keep the SIMDs occupied; r2ag: +8..44 % at K = 3000 / 4096, e.g. bf16
// gs 100 47.6 -> 42.5 us; -10..15 % at K = 2048, hence the threshold).  Otherwise one wave per tile and GPT (8..64, a power of two) from a
// per-row cost fitted to measurements (profiles/round2/r2_rowgroup/r2r_*: 14336 x 4096,
// group sizes 48 / 100, GPT 8..32): tiles x (fixed wave cost 8 + 0.6 per element of a
// lane's pass-1 chunk C = L / (64 / GPT) + 2.3 per 512-element pass-2 sweep).  gpt = 0 if
// the shape does not fit the LDS stage.  rg_gpt / rg_waves override (awq_diag.h).
struct RgPlan {
    int gpt, waves;
};
RgPlan rowgroup_plan(int dtype, int64_t K, int64_t L) {
    RgPlan pl = {0, 1};
    if (dtype != AWQ_DTYPE_BF16 && dtype != AWQ_DTYPE_F16 && dtype != AWQ_DTYPE_F32) return pl;
    const int64_t es = dtype == AWQ_DTYPE_F32 ? 4 : 2;
    // (L = 1: a one-element group's NaN scale keeps the element's own NaN bits — generic kernel)
    if (L < 2 || K <= 0 || K >= ((int64_t)1 << 30) || 8 * L * es > kRgStageBytes) return pl;
    const bool ew = tuning().rg_waves == 1 || tuning().rg_waves == 2;
    if (ew) pl.waves = tuning().rg_waves;
    if (const int v = tuning().rg_gpt) {
        if (v >= 8 && v <= 64 && v % 8 == 0 && v * L * es <= kRgStageMax) {
            pl.gpt = v;
            return pl;
        }
    }
    const int64_t G = (K + L - 1) / L;
    const int64_t whole = (G + 7) / 8 * 8;
    if (!ew && es == 2 && K >= 2560 && whole <= 64 && whole * L * es <= kRgStageMax) {
        pl.gpt = (int)whole;
        pl.waves = 2;
        return pl;
    }
    // long 16-bit rows (>= 96 groups) whose group length is not a multiple of 8 (pass 2 looks
    // parameters up per half-chunk or per element): two waves on tiles of <= 9.6 KB, <= 64
    // groups, the row split into that many tiles of equal multiples of 8 groups (round 4,
    // profiles/round4/r4g/abk_k14336_tiles.txt, r4j/abr_long_rows.txt, r4k/abr.txt: 4096 x
    // 14336 gs 100 -11..22 %, gs 60 -5..11 %, gs 124 -2..3 %, 8192 x 8192 gs 76 -15 %, gs 60
    // -2..5 %; rows of 65-95 groups lost up to 12 % (K = 4096 at gs 60: tiles of 40 + 29
    // groups) and keep one wave, as do L % 8 == 0 sizes — gs 48 / 96 lost up to 30 %)
    if (!ew && es == 2 && G >= 96 && L % 8 != 0 && L >= 56 && L <= 128) {
        const int64_t gmax = min((int64_t)64, 9600 / (L * es) / 8 * 8);
        const int64_t n = (G + gmax - 1) / gmax;                       // tiles per row
        pl.gpt = (int)(((G + n - 1) / n + 7) / 8 * 8);
        pl.waves = 2;
        return pl;
    }
    double best_cost = 0.0;
    for (int gpt = 8; gpt <= 64; gpt *= 2) {
        if (gpt * L * es > kRgStageBytes) break;
        const int64_t tiles = (G + gpt - 1) / gpt;
        const int64_t C = (L + (64 / gpt) - 1) / (64 / gpt);
        const int64_t el = min((int64_t)gpt, G) * L;                  // elements of a full tile
        const double cost = (double)tiles * (8.0 + 0.6 * (double)C + 2.3 * (double)((el + 511) / 512));
        if (pl.gpt == 0 || cost < best_cost) { best_cost = cost; pl.gpt = gpt; }
    }
    return pl;
}
int rowgroup_gpt(int dtype, int64_t K, int64_t L) { return rowgroup_plan(dtype, K, L).gpt; }

hipError_t launch_rowgroup(const void* w, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int symmetric,
                           int32_t* qweight, int32_t* qzeros, uint16_t* scales, int32_t* tensor_q, int32_t* zeros,
                           hipStream_t stream, uint32_t nan_code) {
    const RgPlan pl = rowgroup_plan(dtype, K, L);
    const int gpt = pl.gpt;
    if (gpt == 0 || rows <= 0) return hipErrorInvalidValue;
    const int64_t G = (K + L - 1) / L;
    const int64_t tpr = (G + gpt - 1) / gpt;
    const int nt = 64 * pl.waves;                                      // threads per tile
    const int lgP = min(6, 31 - __builtin_clz((unsigned)(nt / gpt)));  // P = lanes per group: a power of two
    const int P = 1 << lgP;
    const int C = (int)((L + P - 1) / P);
    // the row's last tile when it holds fewer groups: the largest power of two <= nt / its
    // groups lanes per group (<= 64)
    const int64_t ng_last = G - (tpr - 1) * gpt;
    const int lgP_last = min(6, 31 - __builtin_clz((unsigned)(nt / ng_last)));
    const int C_last = (int)((L + (1 << lgP_last) - 1) >> lgP_last);
    const dim3 grid((unsigned)(rows * tpr)), block((unsigned)nt);
    // stage: the tile's elements rounded up to 16 B, + the up-to-16-B alignment skew and the
    // last 8-element vector read past the segment end
    // (sized to the elements a tile can hold: a whole-row tile's groups are rounded up to a
    //  multiple of 8 but its segment ends at K — 8.2 instead of 9.6 KiB for K = 4096 at gs 100
    //  lets 16 two-wave workgroups (8 waves per SIMD) fit a CU's 160 KiB instead of 14;
    //  rg_lds_full = 1 keeps the round-2 sizing for A/B)
    const int64_t es = dtype == AWQ_DTYPE_F32 ? 4 : 2;
    const int64_t stage_el = tuning().rg_lds_full == 1 ? (int64_t)gpt * L : min((int64_t)gpt * L, K);
    size_t lds = (size_t)((stage_el * es + 15) / 16 * 16 + 48);
    // uniform pass 1 (round 4): 16-bit, even K and L, and every tile's P lanes per group split
    // L into P runs of the same even length (so runs start on dwords and the padding of the
    // row's last group can be staged as zeros); the stage then holds the tile's groups whole
    const bool lanes_ok = L % (1 << lgP) == 0 && (L >> lgP) % 2 == 0 &&
                          (ng_last == gpt || (L % (1 << lgP_last) == 0 && (L >> lgP_last) % 2 == 0));
    const int p1u = (es == 2 && K % 2 == 0 && L % 2 == 0 && lanes_ok && tuning().rg_p1u != 1) ? 1 : 0;
    if (p1u) lds = std::max(lds, (size_t)(((7 + min((int64_t)gpt, G) * L) * es + 15) / 16 * 16));
    const bool p1c = tuning().rg_p1 == 2;   // pass 1 by groups (default) / evenly split runs (A/B)
    // the stage by LDS-DMA (default); diagnostics A/B: rg_ldsdma = 1 the round-3 register
    // stage, whose 4-chunk case then feeds pass 2 from its registers unless rg_p2reg = 1
    const int ldsdma = tuning().rg_ldsdma == 1 ? 0 : 1;
    const int p2reg = (tuning().rg_p2reg == 1 || ldsdma) ? 0 : 1;
#define AWQ_RG_GO(Fm, B, S, SP, P1, TQ)                                                                            \
    hipLaunchKernelGGL((awq_rowgroup_kernel<Fm, B, S, SP, P1, TQ>), grid, block, lds, stream, w, rows, K, L, lgP,  \
                       gpt, (uint32_t)tpr, G, C, 1.0f / (float)L, qweight, qzeros, scales, tensor_q, zeros, nan_code, \
                       lgP_last, C_last, p2reg, ldsdma, p1u)
    // (the pass-1 A/B variant is built for the packed outputs only; with tensor_q it takes the default)
#ifdef AWQ_DIAG
#define AWQ_RG_SPLIT(Fm, B, S, SP)                                                                                 \
    do {                                                                                                           \
        if (tensor_q) AWQ_RG_GO(Fm, B, S, SP, false, true);                                                         \
        else if (p1c) AWQ_RG_GO(Fm, B, S, SP, true, false);                                                         \
        else AWQ_RG_GO(Fm, B, S, SP, false, false);                                                                 \
    } while (0)
#else
#define AWQ_RG_SPLIT(Fm, B, S, SP)                                                                                 \
    do {                                                                                                           \
        (void)p1c;                                                                                                  \
        if (tensor_q) AWQ_RG_GO(Fm, B, S, SP, false, true);                                                         \
        else AWQ_RG_GO(Fm, B, S, SP, false, false);                                                                 \
    } while (0)
#endif
#define AWQ_RG(Fm, B, S)                                                                                           \
    if (L % 8 == 0) AWQ_RG_SPLIT(Fm, B, S, 8);                                                                      \
    else if (L % 4 == 0) AWQ_RG_SPLIT(Fm, B, S, 4);                                                                 \
    else AWQ_RG_SPLIT(Fm, B, S, 1)
#define AWQ_RG_FMT(Fm)                                                     \
    switch ((bits == 8 ? 2 : 0) + (symmetric ? 1 : 0)) {                  \
    case 0: AWQ_RG(Fm, 4, false); break;                                   \
    case 1: AWQ_RG(Fm, 4, true); break;                                    \
    case 2: AWQ_RG(Fm, 8, false); break;                                   \
    default: AWQ_RG(Fm, 8, true); break;                                   \
    }
    if (dtype == AWQ_DTYPE_F16) {
        AWQ_RG_FMT(FmtF16)
    } else if (dtype == AWQ_DTYPE_F32) {
        AWQ_RG_FMT(FmtF32)
    } else {
        AWQ_RG_FMT(FmtBF16)
    }
#undef AWQ_RG_FMT
#undef AWQ_RG
#undef AWQ_RG_SPLIT
#undef AWQ_RG_GO
    return hipPeekAtLastError();
}

}  // namespace awq
