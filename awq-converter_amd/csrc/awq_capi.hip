// awq_capi.hip — the extern "C" boundary of libawq_hip.so (declared in include/awq_hip.h).
//
// Validates arguments, picks the kernel, launches on the caller's stream and reports
// errors through a thread-local message.  No allocation, no synchronisation, no global
// mutable state: one instance may be called from many host threads at once (the
// reference's CLI shares one quantizer between its worker threads, main.py:609-621).
#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "awq_internal.h"

namespace {

thread_local std::string g_err;
#ifdef AWQ_DIAG
thread_local awq_tuning g_tuning{};   // awq_diag.h (diagnostics build only)
#endif

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

}  // namespace

namespace awq {
int set_error(int code, const char* msg) { return fail(code, "%s", msg); }   // (awq_stream.hip)
}  // namespace awq

namespace {

int hip_status(hipError_t e, const char* what) {
    if (e == hipSuccess) return AWQ_OK;
    return fail(AWQ_EHIP, "%s: %s", what, hipGetErrorString(e));
}

bool aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

int check_common(int64_t rows, int64_t K, int64_t group_size, int bits) {
    if (bits != 4 && bits != 8) return fail(AWQ_EINVAL, "Unsupported bit width: %d. Supported: 4, 8.", bits);
    if (group_size <= 0) return fail(AWQ_EINVAL, "Group size must be a positive integer: %lld", (long long)group_size);
    if (rows < 0 || K < 0) return fail(AWQ_EINVAL, "negative shape (%lld, %lld)", (long long)rows, (long long)K);
    return AWQ_OK;
}

bool fast_eligible(int dtype, int64_t rows, int64_t K, int64_t group_size) {
    return (dtype == AWQ_DTYPE_BF16 || dtype == AWQ_DTYPE_F16 || dtype == AWQ_DTYPE_F32) &&
           awq::fast_shape_ok(rows, K, group_size);
}

// the row-segment kernel (any group size <= 512, bf16 / fp16 / fp32): 16-B aligned input,
// dword-aligned outputs, segment offsets within int range
bool rowgroup_shape(int dtype, int64_t rows, int64_t K, int64_t group_size) {
    if (awq::tuning().no_rowgroup) return false;   // diagnostics A/B against the generic kernel
    const int gpt = awq::rowgroup_gpt(dtype, K, group_size);
    if (gpt == 0 || rows <= 0 || rows * K >= ((int64_t)1 << 40)) return false;
    const int64_t tiles = rows * (((K + group_size - 1) / group_size + gpt - 1) / gpt);
    return tiles < ((int64_t)1 << 31);                  // one 32-bit grid dimension
}

bool rowgroup_ok(int dtype, int64_t rows, int64_t K, int64_t group_size, const void* w, const void* qweight,
                 const void* qzeros, const void* scales, const void* tensor_q, const void* zeros) {
    return rowgroup_shape(dtype, rows, K, group_size) && aligned(w, 16) && (!qweight || aligned(qweight, 4)) &&
           (!qzeros || aligned(qzeros, 4)) && (!scales || aligned(scales, 2)) && (!tensor_q || aligned(tensor_q, 4)) &&
           (!zeros || aligned(zeros, 4));
}

}  // namespace

#ifdef AWQ_DIAG
namespace awq {
const awq_tuning& tuning() { return g_tuning; }
}  // namespace awq
#endif

extern "C" {

#ifdef AWQ_DIAG
int awq_set_tuning(const awq_tuning* t) {
    g_err.clear();
    if (!t) {
        g_tuning = awq_tuning{};
        return AWQ_OK;
    }
    if (t->max_blocks < 0 || t->tiles_per_wave < 0 || t->rg_waves < 0 || t->rg_waves > 2 || t->rg_gpt < 0 ||
        t->rg_gpt > 64 || t->rg_gpt % 8 != 0)
        return fail(AWQ_EINVAL, "bad tuning values");
    g_tuning = *t;
    return AWQ_OK;
}
#endif

int awq_packs_directly(int dtype, int64_t rows, int64_t K, int64_t group_size) {
    // every kernel writes qweight / qzeros directly since the generic kernel's span rewrite
    (void)rows; (void)K; (void)group_size;
    return (dtype >= AWQ_DTYPE_BF16 && dtype <= AWQ_DTYPE_F64) ? 1 : 0;
}

int awq_abi_version(void) { return AWQ_HIP_ABI_VERSION; }

const char* awq_last_error(void) { return g_err.c_str(); }

int awq_device_check(char* arch, int len) {
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return fail(AWQ_ENODEV, "no HIP device: %s", hipGetErrorString(e));
    hipDeviceProp_t prop;
    e = hipGetDeviceProperties(&prop, dev);
    if (e != hipSuccess) return fail(AWQ_ENODEV, "hipGetDeviceProperties: %s", hipGetErrorString(e));
    if (arch && len > 0) {
        std::strncpy(arch, prop.gcnArchName, (size_t)len - 1);
        arch[len - 1] = 0;
    }
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(AWQ_ENODEV, "libawq_hip.so is built for gfx950 (MI355X); device %d is %s", dev,
                    prop.gcnArchName);
    return AWQ_OK;
}

int awq_ragged_eligible(int dtype, int64_t rows, int64_t K, int64_t group_size) {
    return fast_eligible(dtype, rows, K, group_size) ? 1 : 0;
}

int awq_quantize_groups(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size32,
                        int bits, int symmetric, int32_t* qweight, int32_t* qzeros,
                        uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream) {
    return awq_quantize_groups_ex(w, dtype, rows, K, group_size32, bits, symmetric, 0, qweight, qzeros, scales,
                                  tensor_q, zeros, stream);
}

int awq_quantize_groups_ex(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size32,
                           int bits, int symmetric, int flags, int32_t* qweight, int32_t* qzeros,
                           uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream) {
    g_err.clear();
    const int64_t group_size = group_size32;   // (int32 at the boundary: SURVEY.md §8(b))
    if (int rc = check_common(rows, K, group_size, bits)) return rc;
    if (flags & ~AWQ_Q_SMALL_TENSOR) return fail(AWQ_EINVAL, "unknown flags 0x%x", flags);
    const bool small = (flags & AWQ_Q_SMALL_TENSOR) != 0;
    const uint32_t nan_code = awq::nan_scale_code(dtype, symmetric, small);
    if (dtype < AWQ_DTYPE_BF16 || dtype > AWQ_DTYPE_F64) return fail(AWQ_EINVAL, "unknown dtype code %d", dtype);
    if (!qweight && !qzeros && !scales && !tensor_q && !zeros) return fail(AWQ_EINVAL, "no output requested");
    if (rows * K == 0) return AWQ_OK;
    if (!w) return fail(AWQ_EINVAL, "null input");
    hipStream_t s = (hipStream_t)stream;
    if (fast_eligible(dtype, rows, K, group_size) && aligned(w, 16) && (!qweight || aligned(qweight, 8)) &&
        (!tensor_q || aligned(tensor_q, 16)) && (!zeros || aligned(zeros, 4)) && (!qzeros || aligned(qzeros, 4)) &&
        (!scales || aligned(scales, 2))) {
        awq_tensor_desc d{};
        d.w = w; d.rows = rows; d.K = K; d.qweight = qweight; d.qzeros = qzeros; d.scales = scales;
        d.tensor_q = tensor_q; d.zeros = zeros; d.tile_begin = 0;
        d.tile_count = awq::fast_tiles(rows, K, bits, (int)group_size);
        return hip_status(awq::launch_fast(nullptr, nullptr, &d, 1, d.tile_count, dtype, bits, symmetric,
                                           (int)group_size, (K % group_size) != 0, s, nan_code), "awq fast kernel");
    }
    if (rowgroup_ok(dtype, rows, K, group_size, w, qweight, qzeros, scales, tensor_q, zeros))
        return hip_status(awq::launch_rowgroup(w, dtype, rows, K, group_size, bits, symmetric, qweight, qzeros, scales,
                                               tensor_q, zeros, s, nan_code), "awq row-group kernel");
    // generic path (fp64, groups > 512): one wave per qzeros word's span, packed words direct
    return hip_status(awq::launch_generic(w, dtype, rows, K, group_size, bits, symmetric, tensor_q, scales, zeros,
                                          qweight, qzeros, s, small), "awq generic kernel");
}

int awq_quantize_groups_scaled(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size32, int bits,
                               int symmetric, const float* col_scale, int32_t* qweight, int32_t* qzeros,
                               uint16_t* scales, void* stream) {
    g_err.clear();
    const int64_t group_size = group_size32;
    if (int rc = check_common(rows, K, group_size, bits)) return rc;
    if (dtype < AWQ_DTYPE_BF16 || dtype > AWQ_DTYPE_F32) return fail(AWQ_EINVAL, "dtype must be bf16, fp16 or fp32");
    if (!qweight && !qzeros && !scales) return fail(AWQ_EINVAL, "no output requested");
    if (rows * K == 0) return AWQ_OK;
    if (!w || !col_scale) return fail(AWQ_EINVAL, "null input");
    if (!fast_eligible(dtype, rows, K, group_size) || K % group_size != 0 || K % 8 != 0 || !aligned(w, 16) ||
        !aligned(col_scale, 16) || (qweight && !aligned(qweight, 8)) || (qzeros && !aligned(qzeros, 4)) ||
        (scales && !aligned(scales, 2)))
        return fail(AWQ_EINVAL, "awq_quantize_groups_scaled: shape / group size / alignment outside the one-pass "
                                "kernel (group_size 32-256 dividing K, K %% 8 == 0, 16-B aligned w and col_scale)");
    awq_tensor_desc d{};
    d.w = w; d.rows = rows; d.K = K; d.qweight = qweight; d.qzeros = qzeros; d.scales = scales;
    d.tile_begin = 0;
    d.tile_count = awq::fast_tiles(rows, K, bits, (int)group_size);
    return hip_status(awq::launch_fast(nullptr, nullptr, &d, 1, d.tile_count, dtype, bits, symmetric, (int)group_size,
                                       false, (hipStream_t)stream, awq::nan_scale_code(dtype, symmetric, false), 1, 0,
                                       col_scale),
                      "awq fast kernel (scaled)");
}

int awq_quantize_search(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size32, int bits,
                        int symmetric, int n_grid, int n_candidates, int32_t* qweight, int32_t* qzeros,
                        uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream) {
    return awq_quantize_search_ex(w, dtype, rows, K, group_size32, bits, symmetric, 0, n_grid, n_candidates, qweight,
                                  qzeros, scales, tensor_q, zeros, stream);
}

int awq_quantize_search_ex(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size32, int bits,
                           int symmetric, int flags, int n_grid, int n_candidates, int32_t* qweight, int32_t* qzeros,
                           uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream) {
    g_err.clear();
    const int64_t group_size = group_size32;
    if (int rc = check_common(rows, K, group_size, bits)) return rc;
    if (flags & ~AWQ_Q_SMALL_TENSOR) return fail(AWQ_EINVAL, "unknown flags 0x%x", flags);
    const bool small = (flags & AWQ_Q_SMALL_TENSOR) != 0;
    if (dtype < AWQ_DTYPE_BF16 || dtype > AWQ_DTYPE_F64) return fail(AWQ_EINVAL, "unknown dtype code %d", dtype);
    if (n_grid < 1 || n_candidates < 1 || n_candidates > n_grid)
        return fail(AWQ_EINVAL, "search grid needs 1 <= n_candidates (%d) <= n_grid (%d)", n_candidates, n_grid);
    if (group_size > 512 && K > 512)   // (the small-tensor path uses group = K < group_size)
        return fail(AWQ_EUNSUPPORTED, "scale search supports group_size <= 512 (got %lld)", (long long)group_size);
    if (!qweight && !qzeros && !scales && !tensor_q && !zeros) return fail(AWQ_EINVAL, "no output requested");
    if (rows * K == 0) return AWQ_OK;
    if (!w) return fail(AWQ_EINVAL, "null input");
    hipStream_t s = (hipStream_t)stream;
    if (fast_eligible(dtype, rows, K, group_size) && aligned(w, 16) && (!qweight || aligned(qweight, 8)) &&
        (!tensor_q || aligned(tensor_q, 16)) && (!zeros || aligned(zeros, 4)) && (!qzeros || aligned(qzeros, 4)) &&
        (!scales || aligned(scales, 2))) {
        awq_tensor_desc d{};
        d.w = w; d.rows = rows; d.K = K; d.qweight = qweight; d.qzeros = qzeros; d.scales = scales;
        d.tensor_q = tensor_q; d.zeros = zeros; d.tile_begin = 0;
        d.tile_count = awq::fast_tiles(rows, K, bits, (int)group_size);
        return hip_status(awq::launch_fast(nullptr, nullptr, &d, 1, d.tile_count, dtype, bits, symmetric,
                                           (int)group_size, (K % group_size) != 0, s,
                                           awq::nan_scale_code(dtype, symmetric, small), n_grid, n_candidates),
                          "awq fast search kernel");
    }
    return hip_status(awq::launch_generic(w, dtype, rows, K, group_size, bits, symmetric, tensor_q, scales, zeros,
                                          qweight, qzeros, s, small, n_grid, n_candidates), "awq search kernel");
}

int awq_group_params(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, int bits,
                     int symmetric, double* scales, double* zeros, void* stream) {
    return awq_group_params_ex(w, dtype, rows, K, group_size, bits, symmetric, 0, scales, zeros, stream);
}

int awq_group_params_ex(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, int bits,
                        int symmetric, int flags, double* scales, double* zeros, void* stream) {
    g_err.clear();
    if (flags & ~AWQ_GP_TORCH_GPU) return fail(AWQ_EINVAL, "unknown flags 0x%x", flags);
    if (int rc = check_common(rows, K, group_size, bits)) return rc;
    if (dtype < AWQ_DTYPE_BF16 || dtype > AWQ_DTYPE_F64) return fail(AWQ_EINVAL, "unknown dtype code %d", dtype);
    if (!scales && !zeros) return fail(AWQ_EINVAL, "no output requested");
    if (rows * K == 0) return AWQ_OK;
    if (!w) return fail(AWQ_EINVAL, "null input");
    return hip_status(awq::launch_generic(w, dtype, rows, K, group_size, bits, symmetric, nullptr, nullptr, nullptr,
                                          nullptr, nullptr, (hipStream_t)stream, false, 1, 0, scales, zeros,
                                          (flags & AWQ_GP_TORCH_GPU) != 0),
                      "awq group params");
}

int awq_apply_params(const void* x, int dtype, int64_t rows, int64_t K, int64_t group_size, const double* scales,
                     const double* zeros, int qmin, int qmax, int mode, void* out, void* stream) {
    g_err.clear();
    if (dtype < AWQ_DTYPE_BF16 || dtype > AWQ_DTYPE_F64) return fail(AWQ_EINVAL, "unknown dtype code %d", dtype);
    // the parameters enter both ops at their own (fp32 / fp64) value: one-element semantics
    return awq_apply_params_ex(x, dtype, rows, K, group_size, scales, zeros, qmin, qmax, mode, dtype, dtype,
                               AWQ_APPLY_SCALE_ONE_ELEMENT | AWQ_APPLY_ZERO_ONE_ELEMENT, out, stream);
}

int awq_apply_params_ex(const void* x, int x_dtype, int64_t rows, int64_t K, int64_t group_size,
                        const double* scales, const double* zeros, int qmin, int qmax, int mode, int op1_dtype,
                        int op2_dtype, int flags, void* out, void* stream) {
    g_err.clear();
    if (group_size <= 0) return fail(AWQ_EINVAL, "Group size must be a positive integer: %lld", (long long)group_size);
    if (rows < 0 || K < 0) return fail(AWQ_EINVAL, "negative shape (%lld, %lld)", (long long)rows, (long long)K);
    if (mode != 0 && mode != 1) return fail(AWQ_EINVAL, "unknown mode %d (0 quantize, 1 dequantize)", mode);
    if (x_dtype < AWQ_DTYPE_BF16 || x_dtype > AWQ_DTYPE_U64) return fail(AWQ_EINVAL, "unknown dtype code %d", x_dtype);
    for (int d : {op1_dtype, op2_dtype})
        if (d < AWQ_DTYPE_BF16 || d > AWQ_DTYPE_U8)
            return fail(AWQ_EINVAL, "dtype code %d is not an op dtype (bf16 .. uint8)", d);
    if (mode == 0 && (op1_dtype >= AWQ_DTYPE_I32 || op2_dtype >= AWQ_DTYPE_I32))
        return fail(AWQ_EINVAL, "quantize (mode 0) divides: its ops are floating point");
    constexpr int known = AWQ_APPLY_SCALE_ONE_ELEMENT | AWQ_APPLY_ZERO_ONE_ELEMENT | AWQ_APPLY_SCALE_INT |
                          AWQ_APPLY_ZERO_INT | AWQ_APPLY_SCALE_UNSIGNED | AWQ_APPLY_ZERO_UNSIGNED |
                          AWQ_APPLY_IEEE_CLAMP;
    if (flags & ~known) return fail(AWQ_EINVAL, "unknown flags 0x%x", flags);
    if (((flags & AWQ_APPLY_SCALE_UNSIGNED) && !(flags & AWQ_APPLY_SCALE_INT)) ||
        ((flags & AWQ_APPLY_ZERO_UNSIGNED) && !(flags & AWQ_APPLY_ZERO_INT)))
        return fail(AWQ_EINVAL, "AWQ_APPLY_*_UNSIGNED needs AWQ_APPLY_*_INT");
    if (mode == 0 && qmin > qmax) return fail(AWQ_EINVAL, "qmin %d > qmax %d", qmin, qmax);
    if (rows * K == 0) return AWQ_OK;
    if (!x || !scales || !zeros || !out) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_apply(x, x_dtype, rows, K, group_size, scales, zeros, qmin, qmax, mode, op1_dtype,
                                        op2_dtype, flags, out, (hipStream_t)stream), "awq apply params");
}

int64_t awq_plan_ragged(awq_tensor_desc* descs, int n, int bits, int64_t group_size) {
    g_err.clear();
    if (n < 0 || (n > 0 && !descs)) return fail(AWQ_EINVAL, "bad descriptor array"), -1;
    if (bits != 4 && bits != 8) return fail(AWQ_EINVAL, "Unsupported bit width: %d. Supported: 4, 8.", bits), -1;
    if (!awq::fast_group_size(group_size))
        return fail(AWQ_EUNSUPPORTED, "ragged launches take group_size 32, 64, 128 or 256 (got %lld)",
                    (long long)group_size), -1;
    int64_t total = 0;
    for (int i = 0; i < n; ++i) {
        awq_tensor_desc& d = descs[i];
        if (!fast_eligible(AWQ_DTYPE_BF16, d.rows, d.K, group_size))
            return fail(AWQ_EINVAL, "tensor %d (%lld x %lld) is not eligible for a ragged launch", i,
                        (long long)d.rows, (long long)d.K), -1;
        if (!d.w || !aligned(d.w, 16) || (d.qweight && !aligned(d.qweight, 8)) ||
            (d.tensor_q && !aligned(d.tensor_q, 16)) || (d.zeros && !aligned(d.zeros, 4)) ||
            (d.qzeros && !aligned(d.qzeros, 4)) || (d.scales && !aligned(d.scales, 2)))
            return fail(AWQ_EINVAL, "tensor %d: null or misaligned pointer", i), -1;
        d.tile_begin = total;
        d.tile_count = awq::fast_tiles(d.rows, d.K, bits, (int)group_size);
        total += d.tile_count;
    }
    return total;
}

int64_t awq_plan_block_tensor(const awq_tensor_desc* descs, int n, int64_t total_tiles, int32_t* block_tensor,
                              int64_t len) {
    g_err.clear();
    const int64_t entries = awq::table_entries(total_tiles);
    const int64_t need = entries * awq::kTableEntryInts;   // int32 units
    if (!block_tensor && len == 0) return need;   // size query
    if (!block_tensor || len < need) return fail(AWQ_EINVAL, "block table needs %lld int32", (long long)need), -1;
    if ((uintptr_t)block_tensor % 16) return fail(AWQ_EINVAL, "block table must be 16-B aligned"), -1;
    if (n <= 0 || !descs) return fail(AWQ_EINVAL, "bad descriptor array"), -1;
    awq::TableEntry* tab = (awq::TableEntry*)block_tensor;
    int pair_cur = 0;   // tensor of the current 128-tile pair's first tile (monotone over pairs)
    for (int64_t b = 0; b < entries; ++b) {
        // the entry's tiles t0, t0 + 8, ..., t0 + 56 (awq_internal.h table_index); entries of
        // one 128-tile pair are visited out of tile order, so each steps from the pair's tensor
        const int64_t t = std::min(awq::table_first_tile(b), total_tiles - 1);
        const int64_t last = std::max(t, std::min(t + 8 * (awq::kTableTiles - 1), total_tiles - 1));
        if ((b & 15) == 0) {
            const int64_t tp = std::min((b >> 4) * 128, total_tiles - 1);
            while (pair_cur + 1 < n && descs[pair_cur + 1].tile_begin <= tp) ++pair_cur;
        }
        int cur = pair_cur;
        while (cur + 1 < n && descs[cur + 1].tile_begin <= t) ++cur;
        const bool spans = cur + 1 < n && descs[cur + 1].tile_begin <= last;
        awq::TableEntry e{};
        e.w = descs[cur].w;
        e.tile_begin = descs[cur].tile_begin;
        e.rows = descs[cur].rows;
        e.K = descs[cur].K;
        e.tensor = (int32_t)((uint32_t)cur | (spans ? 0x80000000u : 0u));
        tab[b] = e;
    }
    return need;
}

int awq_ragged_flags(const awq_tensor_desc* descs, int n, int64_t group_size) {
    int flags = 0;
    for (int i = 0; descs && i < n; ++i)
        if (group_size > 0 && descs[i].K % group_size) flags |= AWQ_RAGGED_PADDED;
    return flags;
}

int awq_quantize_ragged(const awq_tensor_desc* descs_device, int n, int64_t total_tiles,
                        const int32_t* block_tensor_device, int dtype, int bits, int symmetric, int64_t group_size,
                        int flags, void* stream) {
    g_err.clear();
    if (bits != 4 && bits != 8) return fail(AWQ_EINVAL, "Unsupported bit width: %d. Supported: 4, 8.", bits);
    if (!awq::fast_group_size(group_size))
        return fail(AWQ_EUNSUPPORTED, "ragged launches take group_size 32, 64, 128 or 256 (got %lld)",
                    (long long)group_size);
    if (dtype != AWQ_DTYPE_BF16 && dtype != AWQ_DTYPE_F16 && dtype != AWQ_DTYPE_F32)
        return fail(AWQ_EINVAL, "ragged launches take bf16, fp16 or fp32 tensors (dtype code %d)", dtype);
    if (flags & ~AWQ_RAGGED_PADDED) return fail(AWQ_EINVAL, "unknown ragged flags 0x%x", flags);
    if (n <= 0 || total_tiles <= 0) return AWQ_OK;
    if (!descs_device) return fail(AWQ_EINVAL, "null descriptor array");
    return hip_status(awq::launch_fast(descs_device, block_tensor_device, nullptr, n, total_tiles, dtype, bits,
                                       symmetric, (int)group_size, (flags & AWQ_RAGGED_PADDED) != 0,
                                       (hipStream_t)stream, awq::nan_scale_code(dtype, symmetric, false)),
                      "awq ragged kernel");
}

int awq_quantize_ragged_search(const awq_tensor_desc* descs_device, int n, int64_t total_tiles,
                               const int32_t* block_tensor_device, int dtype, int bits, int symmetric,
                               int64_t group_size, int flags, int n_grid, int n_candidates, void* stream) {
    g_err.clear();
    if (n_grid < 1 || n_candidates < 1 || n_candidates > n_grid)
        return fail(AWQ_EINVAL, "search grid needs 1 <= n_candidates (%d) <= n_grid (%d)", n_candidates, n_grid);
    if (n_candidates == 1)   // candidate 0 alone is RTN
        return awq_quantize_ragged(descs_device, n, total_tiles, block_tensor_device, dtype, bits, symmetric,
                                   group_size, flags, stream);
    if (bits != 4 && bits != 8) return fail(AWQ_EINVAL, "Unsupported bit width: %d. Supported: 4, 8.", bits);
    if (!awq::fast_group_size(group_size))
        return fail(AWQ_EUNSUPPORTED, "ragged launches take group_size 32, 64, 128 or 256 (got %lld)",
                    (long long)group_size);
    if (dtype != AWQ_DTYPE_BF16 && dtype != AWQ_DTYPE_F16 && dtype != AWQ_DTYPE_F32)
        return fail(AWQ_EINVAL, "ragged launches take bf16, fp16 or fp32 tensors (dtype code %d)", dtype);
    if (flags & ~AWQ_RAGGED_PADDED) return fail(AWQ_EINVAL, "unknown ragged flags 0x%x", flags);
    if (n <= 0 || total_tiles <= 0) return AWQ_OK;
    if (!descs_device) return fail(AWQ_EINVAL, "null descriptor array");
    return hip_status(awq::launch_fast(descs_device, block_tensor_device, nullptr, n, total_tiles, dtype, bits,
                                       symmetric, (int)group_size, (flags & AWQ_RAGGED_PADDED) != 0,
                                       (hipStream_t)stream, awq::nan_scale_code(dtype, symmetric, false), n_grid,
                                       n_candidates),
                      "awq ragged search kernel");
}

int awq_dequantize(const int32_t* tensor_q, const uint16_t* scales, const int32_t* zeros, int64_t rows,
                   int64_t K, int64_t group_size, float* out, void* stream) {
    g_err.clear();
    if (group_size <= 0) return fail(AWQ_EINVAL, "Group size must be a positive integer: %lld", (long long)group_size);
    if (rows * K == 0) return AWQ_OK;
    if (!tensor_q || !scales || !zeros || !out) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_dequant(tensor_q, nullptr, scales, zeros, nullptr, rows, K, group_size, 4, 0,
                                          out, (hipStream_t)stream), "awq dequant kernel");
}

int awq_dequantize_packed(const int32_t* qweight, const int32_t* qzeros, const uint16_t* scales, int64_t rows,
                          int64_t K, int64_t group_size, int bits, int symmetric, float* out, void* stream) {
    g_err.clear();
    if (int rc = check_common(rows, K, group_size, bits)) return rc;
    if (rows * K == 0) return AWQ_OK;
    if (!qweight || !scales || !qzeros || !out) return fail(AWQ_EINVAL, "null argument");
    const int qmin = symmetric ? -(1 << (bits - 1)) : 0;
    return hip_status(awq::launch_dequant(nullptr, qweight, scales, nullptr, qzeros, rows, K, group_size, bits,
                                          qmin, out, (hipStream_t)stream), "awq dequant kernel");
}

int awq_pack_rows(const int32_t* v, int64_t rows, int64_t n, int bits, int qmin, int32_t* packed, void* stream) {
    g_err.clear();
    if (bits != 4 && bits != 8) return fail(AWQ_EINVAL, "Unsupported bit width: %d. Supported: 4, 8.", bits);
    if (rows * n == 0) return AWQ_OK;
    if (!v || !packed) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_pack(v, rows, n, bits, qmin, packed, (hipStream_t)stream), "awq pack");
}

int awq_export_autoawq_gemm(const int32_t* qweight, const int32_t* qzeros, const uint16_t* scales, int64_t N,
                            int64_t K, int64_t group_size, int bits, int32_t* qweight_t, int32_t* qzeros_t,
                            uint16_t* scales_t, void* stream) {
    g_err.clear();
    if (bits != 4) return fail(AWQ_EUNSUPPORTED, "the AutoAWQ GEMM layout is 4-bit only (bits=%d)", bits);
    if (group_size <= 0) return fail(AWQ_EINVAL, "Group size must be a positive integer: %lld", (long long)group_size);
    if (N <= 0 || K <= 0 || N % 8 != 0 || K % 8 != 0 || K % group_size != 0)
        return fail(AWQ_EINVAL, "AutoAWQ GEMM layout needs out_features %% 8 == 0 and in_features %% group_size == 0 "
                                "(N=%lld, K=%lld, group_size=%lld)", (long long)N, (long long)K, (long long)group_size);
    if (!qweight || !qzeros || !scales || !qweight_t || !qzeros_t || !scales_t) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_export_gemm(qweight, qzeros, scales, N, K, group_size, qweight_t, qzeros_t, scales_t,
                                              (hipStream_t)stream), "awq export kernel");
}

int awq_stream_copy(const void* src, void* dst, int64_t bytes, void* stream) {
    g_err.clear();
    if (bytes < 0 || bytes % 16 != 0) return fail(AWQ_EINVAL, "bytes must be a non-negative multiple of 16");
    if (bytes > 0 && (!src || !dst || !aligned(src, 16) || !aligned(dst, 16)))
        return fail(AWQ_EINVAL, "null or misaligned buffer");
    return hip_status(awq::launch_stream_copy(src, dst, bytes, (hipStream_t)stream), "awq stream copy");
}

int awq_stream_ceiling(const void* src, void* dst, int64_t bytes, void* stream) {
    g_err.clear();
    if (bytes < 0 || bytes % 4096 != 0) return fail(AWQ_EINVAL, "bytes must be a non-negative multiple of 4096");
    if (bytes > 0 && (!src || !dst || !aligned(src, 16) || !aligned(dst, 16)))
        return fail(AWQ_EINVAL, "null or misaligned buffer");
    return hip_status(awq::launch_stream_ceiling(src, dst, bytes, (hipStream_t)stream), "awq stream ceiling");
}

int awq_dequant_ceiling(const void* words, void* out, int64_t out_bytes, void* stream) {
    g_err.clear();
    if (out_bytes < 0 || out_bytes % 16 != 0) return fail(AWQ_EINVAL, "out_bytes must be a non-negative multiple of 16");
    if (out_bytes > 0 && (!words || !out || !aligned(words, 4) || !aligned(out, 16)))
        return fail(AWQ_EINVAL, "null or misaligned buffer");
    if (out_bytes / 16 > ((int64_t)1 << 40)) return fail(AWQ_EINVAL, "out_bytes too large");
    return hip_status(awq::launch_dequant_ceiling(words, out, out_bytes, (hipStream_t)stream), "awq dequant ceiling");
}

// ---- activation-aware scale search (include/awq_hip.h awq_act_*) ----
namespace {
int check_act_shape(int dtype, int64_t rows, int64_t K, int64_t group_size) {
    if (dtype != AWQ_DTYPE_BF16 && dtype != AWQ_DTYPE_F16 && dtype != AWQ_DTYPE_F32)
        return fail(AWQ_EUNSUPPORTED, "activation-aware search takes bf16 / fp16 / fp32 weights (dtype code %d)", dtype);
    if (group_size < 8 || group_size > 512 || (group_size & (group_size - 1)) != 0)
        return fail(AWQ_EUNSUPPORTED, "activation-aware search needs a power-of-two group_size in [8, 512] (got %lld)",
                    (long long)group_size);
    if (rows <= 0 || K <= 0 || K % group_size != 0)
        return fail(AWQ_EINVAL, "activation-aware search needs a 2-D [rows, K] weight with K %% group_size == 0 "
                                "(rows=%lld, K=%lld, group_size=%lld)", (long long)rows, (long long)K,
                    (long long)group_size);
    return AWQ_OK;
}
}  // namespace

int awq_act_stats(const void* x, int dtype, int64_t tokens, int64_t K, double* work, float* x_mean, float* x_sq,
                  void* stream) {
    g_err.clear();
    if (dtype != AWQ_DTYPE_BF16 && dtype != AWQ_DTYPE_F16 && dtype != AWQ_DTYPE_F32)
        return fail(AWQ_EUNSUPPORTED, "activations must be bf16 / fp16 / fp32 (dtype code %d)", dtype);
    if (tokens <= 0 || K <= 0) return fail(AWQ_EINVAL, "activations must be a non-empty [tokens, K] matrix");
    if (!x || !work || !x_mean || !x_sq) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_act_stats(x, dtype, tokens, K, work, x_mean, x_sq, (hipStream_t)stream),
                      "awq act stats");
}

int awq_weight_colsum(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, float* gmax_work,
                      double* partial, void* stream) {
    g_err.clear();
    if (int rc = check_act_shape(dtype, rows, K, group_size)) return rc;
    if (!w || !gmax_work || !partial) return fail(AWQ_EINVAL, "null argument");
    if (!aligned(w, 16)) return fail(AWQ_EINVAL, "weights must be 16-B aligned");
    return hip_status(awq::launch_weight_colsum(w, dtype, rows, K, group_size, gmax_work, partial,
                                                (hipStream_t)stream), "awq weight colsum");
}

int awq_column_mean(const double* partial, int64_t nblk, int64_t K, double divisor, float* out, void* stream) {
    g_err.clear();
    if (nblk <= 0 || K <= 0 || !(divisor > 0)) return fail(AWQ_EINVAL, "empty column sum");
    if (!partial || !out) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_colmean(partial, nblk, K, divisor, out, (hipStream_t)stream), "awq column mean");
}

int awq_act_scale_table(const float* x_mean, const float* w_mean, int64_t K, int n_grid, float* table,
                        void* stream) {
    g_err.clear();
    if (n_grid < 1 || n_grid > AWQ_ACT_MAX_GRID)
        return fail(AWQ_EINVAL, "n_grid must be in [1, %d] (got %d)", AWQ_ACT_MAX_GRID, n_grid);
    if (K <= 0) return fail(AWQ_EINVAL, "K must be positive");
    if (!x_mean || !table) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_scale_table(x_mean, w_mean, K, n_grid, table, (hipStream_t)stream),
                      "awq scale table");
}

int awq_act_scale_table_ws(const float* x_mean, const float* w_mean, int64_t K, int n_grid, double* work,
                           float* table, void* stream) {
    g_err.clear();
    if (n_grid < 1 || n_grid > AWQ_ACT_MAX_GRID)
        return fail(AWQ_EINVAL, "n_grid must be in [1, %d] (got %d)", AWQ_ACT_MAX_GRID, n_grid);
    if (K <= 0) return fail(AWQ_EINVAL, "K must be positive");
    if (!x_mean || !table || !work) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_scale_table_ws(x_mean, w_mean, K, n_grid, work, table, (hipStream_t)stream),
                      "awq scale table");
}

int awq_act_recip_table(const float* table, int n_grid, int64_t K, float* rtable, void* stream) {
    g_err.clear();
    if (n_grid < 1 || n_grid > AWQ_ACT_MAX_GRID)
        return fail(AWQ_EINVAL, "n_grid must be in [1, %d] (got %d)", AWQ_ACT_MAX_GRID, n_grid);
    if (K <= 0) return fail(AWQ_EINVAL, "K must be positive");
    if (!table || !rtable) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_recip_table(table, (int64_t)n_grid * K, rtable, (hipStream_t)stream),
                      "awq recip table");
}

int awq_act_search_losses(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, int bits,
                          int symmetric, const float* table, const float* rtable, int n_grid, const float* x_sq,
                          float* part, int64_t part_stride, void* stream) {
    g_err.clear();
    if (bits != 4 && bits != 8) return fail(AWQ_EINVAL, "Unsupported bit width: %d. Supported: 4, 8.", bits);
    if (int rc = check_act_shape(dtype, rows, K, group_size)) return rc;
    if (n_grid < 1 || n_grid > AWQ_ACT_MAX_GRID)
        return fail(AWQ_EINVAL, "n_grid must be in [1, %d] (got %d)", AWQ_ACT_MAX_GRID, n_grid);
    if (part_stride < rows * (K / group_size)) return fail(AWQ_EINVAL, "part_stride smaller than the group count");
    if (!w || !table || !x_sq || !part) return fail(AWQ_EINVAL, "null argument");
    if (!aligned(w, 16) || !aligned(table, 16) || !aligned(x_sq, 16) || !aligned(part, 4) ||
        (rtable && !aligned(rtable, 16)))
        return fail(AWQ_EINVAL, "weights, table, rtable and x_sq must be 16-B aligned");
    return hip_status(awq::launch_act_losses(w, dtype, rows, K, group_size, bits, symmetric, table, rtable, n_grid,
                                             x_sq, part, part_stride, (hipStream_t)stream), "awq act losses");
}

int awq_act_search_select(const float* part, int n_grid, int64_t part_stride, const float* table, int64_t K,
                          double* work, double* losses, int32_t* best, float* s_best, void* stream) {
    g_err.clear();
    if (n_grid < 1 || n_grid > AWQ_ACT_MAX_GRID)
        return fail(AWQ_EINVAL, "n_grid must be in [1, %d] (got %d)", AWQ_ACT_MAX_GRID, n_grid);
    if (part_stride <= 0 || K <= 0) return fail(AWQ_EINVAL, "empty search");
    if (!part || !table || !work) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_act_select(part, n_grid, part_stride, table, K, work, losses, best, s_best,
                                             (hipStream_t)stream), "awq act select");
}

int awq_apply_input_scale(const void* w, int dtype, int64_t rows, int64_t K, const float* s, void* out,
                          void* stream) {
    g_err.clear();
    if (dtype != AWQ_DTYPE_BF16 && dtype != AWQ_DTYPE_F16 && dtype != AWQ_DTYPE_F32)
        return fail(AWQ_EUNSUPPORTED, "input scaling takes bf16 / fp16 / fp32 weights (dtype code %d)", dtype);
    if (rows < 0 || K < 0) return fail(AWQ_EINVAL, "negative shape");
    if (rows * K == 0) return AWQ_OK;
    if (!w || !s || !out) return fail(AWQ_EINVAL, "null argument");
    return hip_status(awq::launch_apply_scale(w, dtype, rows, K, s, out, (hipStream_t)stream), "awq apply scale");
}

int awq_selftest(int which, unsigned long long* result, void* stream) {
    g_err.clear();
    if (!result) return fail(AWQ_EINVAL, "null result pointer");
    if (which == 1) return hip_status(awq::launch_selftest_mquot(result, (hipStream_t)stream), "awq selftest");
    if (which != 0 && which != 2) return fail(AWQ_EINVAL, "unknown self-test %d", which);
    return hip_status(awq::launch_selftest(which, result, (hipStream_t)stream), "awq selftest");
}

}  // extern "C"
