/*
 * awq_hip.h — C ABI of libawq_hip.so, the MI355X (gfx950) group quantizer.
 *
 * The reference (shanefitch/AWQ-Converter) has no FFI: its hot path is the Python
 * method AWQQuantizer._quantize_per_group (src/awq_quantizer/quantization/awq.py:286-374),
 * reached from AWQQuantizer.quantize (awq.py:376-433) and from the CLI's
 * quantize_tensor_batch (src/awq_quantizer/main.py:374).  These entry points replace
 * that method's arithmetic; the drop-in Python class (awq-converter_amd/awq_quantizer/
 * quantization/awq.py) binds them with ctypes.  See INTEGRATION.md.
 *
 * Conventions (all entry points):
 *   - plain pointers and sizes; every pointer argument is DEVICE memory allocated by the
 *     caller unless stated otherwise; the library never allocates or frees device memory
 *     and keeps no global mutable state (re-entrant; one stream per call);
 *   - `stream` is a hipStream_t (NULL = legacy default stream); launches are asynchronous
 *     on that stream, nothing synchronises;
 *   - return 0 on success, an AWQ_E* code otherwise; awq_last_error() (thread-local)
 *     then holds a message.  Invalid arguments are reported before anything is launched.
 *
 * Layout: the input is [rows, K] row-major (the reference's dim 0 = rows, remaining dims
 * flattened = K, awq.py:306-320).  Groups are `group_size` consecutive elements along K;
 * a tail group shorter than group_size is zero-padded for its min/max (awq.py:337-339).
 * G = ceil(K / group_size).
 *
 * Outputs (each may be NULL when not wanted; at least one must be non-NULL):
 *   scales    fp16 bits [rows, G]            (awq.py:411, value = fp16(scale))
 *   zeros     int32     [rows, G]            (awq.py:412, reference zero_points)
 *   tensor_q  int32     [rows, K]            (awq.py:410, reference tensor_q)
 *   qweight   int32     [rows, ceil(K*bits/32)]  packed: element k of a row sits in word
 *             k/(32/bits), bits [bits*(k%(32/bits)), +bits), value (q - qmin) & (2^bits-1)
 *   qzeros    int32     [rows, ceil(G*bits/32)]  same packing of the zero points
 * NaN groups/elements follow the reference: int32 outputs are INT32_MIN (x86 cvtt), packed
 * fields hold (INT32_MIN - qmin) & mask, and NaN scales carry the reference's own bits
 * (awq.py:192-205 -> 327/352 -> 411 on x86 torch CPU; pinned by tests/golden/golden_nan.*):
 *   bf16 input 0x7E00; fp16 input 0x7FFF (small-tensor path: 0xFE00 asymmetric, 0x7E00
 *   symmetric); fp32 / fp64 input 0xFFFF when the group holds a NaN, 0xFE00 when the NaN is
 *   inf - inf (an asymmetric group of all +inf or all -inf); a one-element group keeps its
 *   element's NaN (sign — set when symmetric — and top 10 mantissa bits, quiet bit set).
 */
#ifndef AWQ_HIP_H
#define AWQ_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AWQ_HIP_ABI_VERSION 17

/* dtype codes of the input weights (torch dtypes the reference accepts, awq.py:397);
 * the integer codes only in awq_apply_params_ex (integer tensors such as quantize()'s int32
 * tensor_q, and integer ops): I32 .. U8 as tensor and op dtypes, BOOL / U16 / U32 / U64 as
 * tensor dtypes only (ABI 17) */
enum { AWQ_DTYPE_BF16 = 0, AWQ_DTYPE_F16 = 1, AWQ_DTYPE_F32 = 2, AWQ_DTYPE_F64 = 3, AWQ_DTYPE_I32 = 4,
       AWQ_DTYPE_I64 = 5, AWQ_DTYPE_I16 = 6, AWQ_DTYPE_I8 = 7, AWQ_DTYPE_U8 = 8, AWQ_DTYPE_BOOL = 9,
       AWQ_DTYPE_U16 = 10, AWQ_DTYPE_U32 = 11, AWQ_DTYPE_U64 = 12 };

/* status codes */
enum { AWQ_OK = 0, AWQ_EINVAL = 1, AWQ_EUNSUPPORTED = 2, AWQ_EHIP = 3, AWQ_ENODEV = 4 };

/* One tensor of a ragged (multi-tensor) launch.  Same meaning as the awq_quantize_groups
 * arguments.  tile_begin / tile_count are filled by awq_plan_ragged. */
typedef struct awq_tensor_desc {
    const void* w;
    int64_t rows;
    int64_t K;
    int32_t* qweight;
    int32_t* qzeros;
    uint16_t* scales;
    int32_t* tensor_q;
    int32_t* zeros;
    int64_t tile_begin;
    int64_t tile_count;
} awq_tensor_desc;

/* ABI version (AWQ_HIP_ABI_VERSION). */
int awq_abi_version(void);

/* Message of the last failing call on this thread ("" if none). */
const char* awq_last_error(void);

/* AWQ_OK if the current HIP device is a gfx950 (MI355X), AWQ_ENODEV otherwise.
 * Host-only query; writes the device's gcnArchName into arch (if arch != NULL, len > 0). */
int awq_device_check(char* arch, int len);

/* Quantize one [rows, K] tensor (replaces awq.py:286-374 incl. the small-tensor
 * path awq.py:130-171, which a caller expresses as group_size = K).
 * bits in {4, 8}; symmetric selects qmin/qmax per awq.py:114-128.  Kernels, all with the
 * same results:
 *   bf16 / fp16 / fp32, group_size in {32, 64, 128, 256}, K % group_size == 0 or K % 8 == 0
 *     (padded rows, awq.py:337-339): the streaming kernel;
 *   bf16 / fp16 with any other group_size <= 512 (fp32: <= 256), or any K: the row-segment
 *     kernel (packed outputs written directly);
 *   everything else (fp64, larger groups): the generic kernel (one wave per span of groups
 *     sharing a qzeros word; packed outputs written directly too, since round 2).
 * tensor_q / zeros are optional outputs on every path. */
int awq_quantize_groups(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size,
                        int bits, int symmetric, int32_t* qweight, int32_t* qzeros,
                        uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream);

/* flags of the _ex entry points: the call is the small-tensor path (awq.py:297-300 ->
 * _calculate_scale_zp awq.py:130-171, numel < group_size, expressed as group_size = K): its
 * input-dtype scales reach fp16 directly (awq.py:411) instead of through the fp32 [R, G]
 * buffer of awq.py:327 — only the bits of NaN scales differ (fp16 input, see above). */
#define AWQ_Q_SMALL_TENSOR 1

/* awq_quantize_groups with flags (0 = awq_quantize_groups). */
int awq_quantize_groups_ex(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size,
                           int bits, int symmetric, int flags, int32_t* qweight, int32_t* qzeros,
                           uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream);

/* Opt-in per-group clip search (scale_method="search"; no reference counterpart: the
 * reference stores scale_method but never uses it, awq.py:66,111-112 — SURVEY.md §8a).
 * Same inputs/outputs as awq_quantize_groups.  For every group the min/max (after the
 * symmetric abs-max, awq.py:196-199) are shrunk by alpha_i = (n_grid - i) / n_grid,
 * i = 0 .. n_candidates-1, each candidate's scale/zero point taken exactly as RTN
 * (awq.py:202-211), and the candidate with the smallest sum of squared errors between
 * the group and its dequantization (awq.py:459-539 arithmetic) is kept; ties and NaN/inf
 * groups keep i = 0, i.e. the RTN result bit-exactly.  1 <= n_candidates <= n_grid.
 * The squared error is summed in fp32 (fp64 for fp64 input) in one canonical order, so
 * every kernel gets the same bits: chunk c = the group's elements 8c .. 8c+7 summed in
 * order, then a pairwise tree over 64 chunk slots, adjacent pairs first (empty slots = 0):
 * group_size <= 512.
 * tensor_q / zeros are optional outputs (no staging buffers needed). */
int awq_quantize_search(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size, int bits,
                        int symmetric, int n_grid, int n_candidates, int32_t* qweight, int32_t* qzeros,
                        uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream);
/* awq_quantize_search with flags (AWQ_Q_SMALL_TENSOR). */
int awq_quantize_search_ex(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size, int bits,
                           int symmetric, int flags, int n_grid, int n_candidates, int32_t* qweight,
                           int32_t* qzeros, uint16_t* scales, int32_t* tensor_q, int32_t* zeros, void* stream);

/* The reference's per-group scale and zero point (_compute_scale_zp_for_group, awq.py:173-213)
 * in the input dtype's own arithmetic, as exact doubles [rows, G] (bf16 / fp16 / fp32 / fp64
 * values; NaN groups give NaN).  What _quantize_per_group stores in its fp32 scale / zero
 * tensors (awq.py:327-328, 352-353) is these values rounded to fp32; the small-tensor path
 * (awq.py:130-171) is group_size = K.  Either output may be NULL. */
int awq_group_params(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, int bits,
                     int symmetric, double* scales, double* zeros, void* stream);

/* (ABI 17) awq_group_params with flags.  AWQ_GP_TORCH_GPU: the same lines as torch's GPU kernels
 * evaluate them (the reference quantizer with device="cuda"): the scale's division by the Python
 * int qmax - qmin is a product with the reciprocal RN(1 / (qmax - qmin)) in the op's compute
 * type (ATen's GPU division by a CPU scalar), and a zero point clamped from -0 is +0 (the GPU
 * clamp's IEEE maximum).  flags = 0: awq_group_params (torch's CPU semantics). */
#define AWQ_GP_TORCH_GPU 1
int awq_group_params_ex(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, int bits,
                        int symmetric, int flags, double* scales, double* zeros, void* stream);

/* Elementwise with caller-given parameters per group (scales / zeros double [rows, G], used
 * in the op's compute type — fp32, fp64 for fp64 inputs — unrounded to the input dtype, as
 * torch's CPU kernels use a 0-d operand; group_size 1 = one parameter per element), result
 * in the input dtype (out [rows, K]):
 *   mode 0: clamp(round(RN(RN(x / s) + z)), qmin, qmax)   (_quantize_tensor, awq.py:215-250;
 *           NaN stays NaN)
 *   mode 1: RN(RN(x - z) * s)                             (_dequantize_tensor, awq.py:252-284) */
int awq_apply_params(const void* x, int dtype, int64_t rows, int64_t K, int64_t group_size, const double* scales,
                     const double* zeros, int qmin, int qmax, int mode, void* out, void* stream);

/* awq_apply_params_ex flags: the scale / zero point is a one-element operand of the
 * reference's expression (any shape of numel 1) evaluated by torch's CPU kernels (a
 * reference quantizer with device="cpu"; on CUDA a one-element device tensor is converted to
 * the op dtype like any other operand: leave the flag off) */
#define AWQ_APPLY_SCALE_ONE_ELEMENT 1
#define AWQ_APPLY_ZERO_ONE_ELEMENT 2
/* (ABI 17) the scales / zeros array holds int64 values, not doubles (an integer or bool
 * parameter, exact beyond 2^53); _UNSIGNED: those 64-bit words are uint64 values */
#define AWQ_APPLY_SCALE_INT 4
#define AWQ_APPLY_ZERO_INT 8
#define AWQ_APPLY_SCALE_UNSIGNED 16
#define AWQ_APPLY_ZERO_UNSIGNED 32
/* (ABI 17) mode 0's clamp as torch's GPU kernels evaluate it: clamp(-0, 0, qmax) = +0 (IEEE
 * maximum); without it the -0 stays, as torch's CPU clamp keeps an operand equal to the bound.
 * Together with the ONE_ELEMENT flags left off: the reference quantizer with device="cuda". */
#define AWQ_APPLY_IEEE_CLAMP 64

/* The same two ops with torch's type promotion (ABI 15; replaces awq.py:245 and awq.py:282 for
 * parameters of any dtype, e.g. bf16 weights with fp32 per-channel scales, or quantize()'s
 * int32 tensor_q dequantized with fp16 scales):
 *   mode 0: a = x / s in op1_dtype; t = a + z in op2_dtype; round, clamp(qmin, qmax)
 *   mode 1: a = x - z in op1_dtype; t = a * s in op2_dtype
 * op1_dtype / op2_dtype are torch's result dtypes of the two ops (the caller's promotion);
 * out [rows, K] is op2_dtype.  x_dtype may be any integer code too (int64 / int32 / int16 /
 * int8 / uint8 / bool / uint16 / uint32 / uint64 tensors: the reference evaluates awq.py:245 and
 * :282 for any tensor dtype), the op dtypes I32 .. U8 (mode 1 only; integer ops wrap at their
 * width like torch's integer kernels).  Each op: operands converted to its dtype (c10::convert:
 * a float to bf16 / fp16 through fp32; an integer to a float dtype as RN_f32 of the exact
 * integer, then RN to bf16 / fp16, to fp64 directly; to an integer dtype by truncation), fp32
 * math for bf16 / fp16 / fp32 (fp64 for fp64), result rounded to the dtype — except that a
 * parameter flagged AWQ_APPLY_*_ONE_ELEMENT enters a bf16 / fp16 op at its own value in fp32
 * (ATen's reduced-float CPU kernels read a one-element operand's original value).  scales /
 * zeros: the parameters' exact values as doubles (or int64 / uint64 words, AWQ_APPLY_*_INT),
 * [rows, G] as in awq_apply_params (group_size 1 = one per element).
 * awq_apply_params(x, D, ...) = awq_apply_params_ex(x, D, ..., D, D, both flags, ...). */
int awq_apply_params_ex(const void* x, int x_dtype, int64_t rows, int64_t K, int64_t group_size,
                        const double* scales, const double* zeros, int qmin, int qmax, int mode, int op1_dtype,
                        int op2_dtype, int flags, void* out, void* stream);

/* 1 if awq_quantize_groups writes qweight / qzeros for this dtype / shape without the int32
 * tensor_q / zeros staging buffers.  Since round 2 every kernel does (the generic kernel packs
 * per span of groups), so this is 1 for every supported dtype; kept for ABI compatibility. */
int awq_packs_directly(int dtype, int64_t rows, int64_t K, int64_t group_size);

/* True (1) if a tensor of this dtype/shape is eligible for awq_quantize_ragged. */
int awq_ragged_eligible(int dtype, int64_t rows, int64_t K, int64_t group_size);

/* HOST helper: fills descs[i].tile_begin / tile_count (host array) for a ragged launch
 * and returns the total tile count (< 0 on error).  All tensors must be eligible for this
 * group_size (32, 64, 128 or 256; a tile is 2048 elements = 2048 / group_size groups). */
int64_t awq_plan_ragged(awq_tensor_desc* descs_host, int n, int bits, int64_t group_size);

/* Tiles per entry of the ragged launch's tensor table (awq_plan_block_tensor); the kernel's
 * workgroup size is the library's own business (one 64-lane wave per tile). */
#define AWQ_BLOCK_TILES 8

/* HOST helper: the ragged launch's tensor table, one 64-B entry per AWQ_BLOCK_TILES tiles
 * (opaque to the caller: 16 int32 each; ceil(total_tiles / 128) * 16 entries): the input
 * pointer, first tile and shape of the tensor holding the entry's first tile (so a wave
 * issues its loads after one scalar load) and its descriptor index, with bit 31 set when
 * the entry's tiles span more than one tensor (a wave then steps forward from there to its
 * own).  An entry's tiles are the 8 tiles of one XCD in a 64-tile window (t0 + 8 j), so
 * each 128-B line of the table is read by one XCD.  Returns the number of int32
 * written (< 0 on error: len too small, or block_tensor_host not 16-B aligned);
 * block_tensor_host = NULL with len = 0 returns the length needed without writing.
 * descs_host as planned by awq_plan_ragged (the pointers are the device pointers the
 * launch will read). */
int64_t awq_plan_block_tensor(const awq_tensor_desc* descs_host, int n, int64_t total_tiles,
                              int32_t* block_tensor_host, int64_t len);

/* flags of awq_quantize_ragged: some tensor has K % group_size != 0 (padded rows: the
 * kernel instance with the row-tile path; the others are built without it) */
#define AWQ_RAGGED_PADDED 1

/* HOST helper: the awq_quantize_ragged flags a descriptor array needs. */
int awq_ragged_flags(const awq_tensor_desc* descs_host, int n, int64_t group_size);

/* Quantize n eligible tensors of one dtype (AWQ_DTYPE_BF16, _F16 or _F32) in ONE
 * launch (replaces the CLI's per-tensor loop, main.py:353-392).  descs_device: device copy
 * of the array planned by awq_plan_ragged with the same bits and group_size (the caller
 * uploads it; reusable across calls).  block_tensor_device: optional device copy of the
 * awq_plan_block_tensor table (NULL: each wave searches the descriptors). */
int awq_quantize_ragged(const awq_tensor_desc* descs_device, int n, int64_t total_tiles,
                        const int32_t* block_tensor_device, int dtype, int bits, int symmetric, int64_t group_size,
                        int flags, void* stream);

/* awq_quantize_ragged with the opt-in clip search of awq_quantize_search (round 5): the same
 * bits as awq_quantize_search on every tensor of the batch, one launch for a model's tensor
 * set.  1 <= n_candidates <= n_grid (n_candidates = 1: plain RTN, awq_quantize_ragged). */
int awq_quantize_ragged_search(const awq_tensor_desc* descs_device, int n, int64_t total_tiles,
                               const int32_t* block_tensor_device, int dtype, int bits, int symmetric,
                               int64_t group_size, int flags, int n_grid, int n_candidates, void* stream);

/* AutoAWQ "GEMM" layout (the reference has no packed format): from
 * this library's row-major packed 4-bit results of an [N = out_features, K = in_features]
 * weight (qweight [N, K/8], qzeros [N, ceil(G/8)], scales fp16 [N, G], G = K / group_size)
 * to qweight_t int32 [K, N/8], qzeros_t int32 [G, N/8], scales_t fp16 [G, N], packed along
 * N with AWQ_ORDER {0,2,4,6,1,3,5,7} (nibble i of word c = column 8c + AWQ_ORDER[i]).
 * bits must be 4; N % 8 == 0; K % group_size == 0. */
int awq_export_autoawq_gemm(const int32_t* qweight, const int32_t* qzeros, const uint16_t* scales, int64_t N,
                            int64_t K, int64_t group_size, int bits, int32_t* qweight_t, int32_t* qzeros_t,
                            uint16_t* scales_t, void* stream);

/* Measurement helper: copy `bytes` (multiple of 16, 16-B aligned buffers) with the
 * quantizer's memory structure (one wave per 4 KiB, 16-B nt loads/stores); bench.py
 * quotes the kernel against this copy's rate. */
int awq_stream_copy(const void* src, void* dst, int64_t bytes, void* stream);

/* Measurement helper: the quantizer's read-dominant memory structure without its
 * arithmetic — reads `bytes` (multiple of 4096, 16-B aligned) in 4 KiB waves and writes
 * bytes / 4 to dst (one 16-B store per lane per 4 KiB).  bench.py quotes the kernel
 * against this stream's (read + write) rate. */
int awq_stream_ceiling(const void* src, void* dst, int64_t bytes, void* stream);

/* Measurement helper (ABI 17): awq_dequantize_packed's memory structure for 4-bit outputs without
 * its arithmetic — reads out_bytes / 8 of `words` (4-B aligned; 4-B nt loads, a lane pair per
 * dword) and writes out_bytes (16-B aligned, multiple of 16) as 16-B nt stores, 1 KiB per wave
 * instruction: the 1 : 8 read : write stream the dequantize kernel is quoted against
 * (scripts/dq_ceiling_bench.py). */
int awq_dequant_ceiling(const void* words, void* out, int64_t out_bytes, void* stream);

/* Reference dequantize (awq.py:459-539): out fp32 [rows, K] =
 * fp16( fp16(tensor_q - zeros) * scales ) per element.  A NaN result widens its fp16 bits,
 * except in the last n % 8 elements of a group of n = min(group_size, K - g group_size)
 * elements, where it is 0x7FFFFFFF (the reference's fp16 -> fp32 copy, awq.py:527/531). */
int awq_dequantize(const int32_t* tensor_q, const uint16_t* scales, const int32_t* zeros,
                   int64_t rows, int64_t K, int64_t group_size, float* out, void* stream);

/* Same from the packed outputs (qweight/qzeros/scales) of the same bits/symmetric. */
int awq_dequantize_packed(const int32_t* qweight, const int32_t* qzeros, const uint16_t* scales,
                          int64_t rows, int64_t K, int64_t group_size, int bits, int symmetric,
                          float* out, void* stream);

/* Pack int32 values [rows, n] into [rows, ceil(n*bits/32)] words ((v - qmin) & mask). */
int awq_pack_rows(const int32_t* v, int64_t rows, int64_t n, int bits, int qmin, int32_t* packed,
                  void* stream);

/* ---- Host streaming pipeline ----------------------------------
 * Replaces the CLI's read -> quantize -> collect loop (reference main.py:216-392, which
 * loads every file whole and then quantizes tensor by tensor): tensors are pread from their
 * safetensors files straight into pinned staging slots by native reader threads, copied to
 * HBM on an H2D stream, quantized on the compute stream by one ragged launch per dtype and
 * batch (awq_quantize_ragged; shapes it does not take: awq_quantize_groups_ex per tensor),
 * and their outputs copied back on a D2H stream — read, H2D, kernels and D2H of neighbouring
 * batches overlap, with no per-tensor work in the host language.  A 2-D tensor larger than
 * what is left of a slot is split by rows (rows quantize independently, awq.py:332-368), so
 * slots stay small (pipeline fill) whatever the largest tensor.
 *
 * Caller-owned memory: staging slots (pinned host + device), per-slot descriptor tables
 * (pinned host + device, awq_stream_table_bytes each), every item's device outputs and, when
 * its results are wanted on the host, a pinned host range of the same size.  Streams (ABI
 * 14): a stream left NULL in the config is created by the pipeline (non-blocking) and
 * destroyed by awq_stream_end, on its submitter thread while the readers fill the first
 * slots; a non-NULL stream is the caller's.  The submitter first joins the device's
 * first-use warm-up (awq_runtime_warmup below), or runs it if nobody started it. */

/* HIP's first-use costs of a process on a device — its first hardware queue (~85 ms on
 * MI355X), first large copy (~7 ms) and the code object of the quantize kernels (~9 ms) —
 * paid on a native thread of its own: three non-blocking streams (kept for the device's
 * first pipeline, whose NULL config streams they become), one 8 MiB H2D, copy kernel and
 * D2H (buffers freed after).  Returns at once; a later call for the same device does nothing.
 * A CLI starts it as soon as it knows its device, so the costs overlap its host-side setup
 * (file index, planning, pinned allocations). */
int awq_runtime_warmup(int device);

/* Join the device's warm-up if it was started (else return at once); *seconds (may be NULL)
 * = its duration.  Call it before the process exits if the warm-up may still run. */
int awq_runtime_warmup_wait(int device, double* seconds);

/* (awq_stream_*, continued)
 *
 * Bounded output memory (round 4): the caller may place the items' device outputs and host
 * ranges in two RINGS that later items reuse, with two per-item gates:
 *   dev_gate  = g > 0: the kernels writing this item's outputs first wait (on the compute
 *               stream, no host block) for the D2H of items [0, g) — the earlier items whose
 *               device ranges this item's overlap;
 *   host_gate = g > 0: the D2H into this item's host range waits until the caller has
 *               released items [0, g) (awq_stream_release: it no longer reads their host
 *               results, e.g. once their output files are written).
 * awq_stream_plan gives the batch of every item's first and last piece before the start,
 * so the caller can place the rings; awq_stream_start rejects a dev_gate that would wait
 * for a D2H of the same or a later batch, and a host_gate > the item's index.  A caller
 * that releases only what the items before a batch let it release must size the host ring
 * so that a batch's gate never needs that batch's own items (awq_stream_plan).
 *
 * scale_method="search" (awq_quantize_search) runs through the pipeline too: config
 * search_candidates > 0 makes every piece's launch awq_quantize_search_ex with
 * search_grid / search_candidates (rows are independent, so a row split gives the bits of
 * the whole-tensor call). */
#define AWQ_STREAM_MAX_BATCH_ITEMS 4096

typedef struct awq_stream_item {
    int32_t fd;          /* readable file descriptor (pread) */
    int32_t dtype;       /* AWQ_DTYPE_* of the stored tensor */
    int64_t offset;      /* byte offset of the tensor's data in the file */
    int64_t rows, K;     /* awq.py:306-320: rows = dim 0 (1 for a 1-D tensor), K = the rest */
    int32_t* qweight;    /* device outputs (any may be NULL), as awq_quantize_groups */
    int32_t* qzeros;
    uint16_t* scales;
    int32_t* tensor_q;
    int32_t* zeros;
    void* dev_out;       /* D2H of [dev_out, dev_out + out_bytes) (the item's outputs, laid out */
    void* host_out;      /* by the caller inside that range) into pinned host_out; NULL: none */
    int64_t out_bytes;
    void* dev_out2;      /* a second range (e.g. the fp16 scales, kept in a buffer of their */
    void* host_out2;     /* own dtype), NULL: none */
    int64_t out_bytes2;
    int32_t dev_gate;    /* 0: none; see "Bounded output memory" above */
    int32_t host_gate;   /* 0: none */
} awq_stream_item;

typedef struct awq_stream_config {
    int32_t bits, symmetric, group_size, readers;   /* readers: pread threads (>= 1) */
    int32_t nslots;                                 /* >= 2 */
    int32_t trace_batches;                          /* capacity of `trace`, in batches */
    int32_t search_grid, search_candidates;         /* scale_method="search"; 0 candidates = RTN */
    int64_t slot_bytes;          /* input bytes per staging slot, multiple of 4096 */
    int64_t first_batch_bytes;   /* capacity of the first batch (<= slot_bytes; 0 = slot_bytes) */
    void* host_staging;          /* pinned host, nslots * (awq_stream_table_bytes(slot_bytes) +
                                    slot_bytes): each slot = its batch's descriptor / tensor-table
                                    area, then its input; one H2D carries both */
    void* dev_staging;           /* device, the same size */
    void* compute_stream;        /* NULL: the pipeline's own (see above) */
    void* h2d_stream;
    void* d2h_stream;
    double* trace;               /* optional (NULL = off): AWQ_STREAM_TRACE_FIELDS doubles per
                                    batch, seconds from the start, filled by awq_stream_end:
                                    first read began, last read ended, H2D enqueued, kernels
                                    enqueued, D2H enqueued (host clock); H2D done, kernels done,
                                    D2H done (HIP event clock, from an event on the H2D stream,
                                    offset to the host clock at its recording); seconds spent
                                    inside the H2D call and
                                    inside the D2H calls; seconds of the batch's host planning,
                                    of waiting for the slot's previous kernels, of the ragged
                                    launches and of the per-tensor launches;
                                    batches past trace_batches are not traced. */
} awq_stream_config;

#define AWQ_STREAM_TRACE_FIELDS 14

typedef struct awq_stream_stats {
    int64_t batches, pieces, bytes_read;
    double wall_s;               /* start -> last batch's outputs ready */
    double read_busy_s;          /* summed over reader threads */
    double wait_read_s;          /* submitter waiting for a batch's reads */
    double wait_slot_s;          /* submitter waiting for a slot's previous kernels */
    double wait_release_s;       /* submitter waiting for host-ring releases (host_gate) */
    double prepare_s;            /* submitter's device preparation (streams, first-use warm-up) */
} awq_stream_stats;

/* Per-slot descriptor / tensor-table bytes (descriptors + tensor tables of up to
 * AWQ_STREAM_MAX_BATCH_ITEMS pieces): the head of every staging slot; a multiple of 4096. */
int64_t awq_stream_table_bytes(int64_t slot_bytes);

/* HOST only: the batches awq_stream_start would plan for these items and this config
 * (same slot_bytes / first_batch_bytes), without starting anything: first_batch[i] /
 * last_batch[i] = the batch of item i's first / last piece (an item without elements:
 * the batch that completes it, both).  Returns the number of batches (< 0: error). */
int64_t awq_stream_plan(const awq_stream_item* items, int n, const awq_stream_config* cfg, int32_t* first_batch,
                        int32_t* last_batch);

/* Plan the batches and start the pipeline on its own native threads; returns at once.
 * *handle receives the pipeline (awq_stream_end frees it).  Items are processed in order. */
int awq_stream_start(const awq_stream_item* items, int n, const awq_stream_config* cfg, void** handle);

/* The caller no longer reads the host results of items [0, items) (monotone: a smaller
 * count than an earlier call is ignored); wakes a D2H waiting on a host_gate. */
int awq_stream_release(void* handle, int32_t items);

/* Number of batches of a started pipeline. */
int64_t awq_stream_batches(void* handle);

/* Block until batch b's outputs are ready (on the host for items with host_out, on the
 * device otherwise); [*first_item, *end_item) = the items whose last piece is in batch b.
 * Returns the pipeline's first error (its message in awq_last_error), if any. */
int awq_stream_wait(void* handle, int64_t batch, int32_t* first_item, int32_t* end_item);

/* Wait for the whole pipeline, join its threads, release the handle; stats may be NULL.
 * Returns the first error of the pipeline.  Batches not yet copied back when it is called
 * (the caller stopped early) are cancelled rather than copied into host ranges the caller
 * may still be reading. */
int awq_stream_end(void* handle, awq_stream_stats* stats);

/* ---- Activation-aware per-input-channel scale search (scale_method="awq") ----------
 * Not in the reference (it stores scale_method, awq.py:66, and collects no activations;
 * parity unpinned).  AutoAWQ's published search (third-party,
 * not vendored in the reference) restated with a per-element loss, for one "layer group"
 * of n >= 1 linears W_j [R_j, K] that read the same input x [tokens, K]:
 *
 *   x_mean[k] = fp32(sum_t |x[t,k]| / T),  x_sq[k] = fp32(sum_t x[t,k]^2 / T)
 *       (awq_act_stats; sums in fp64: t ascending inside 32-token sub-blocks, the
 *        sub-blocks ascending inside 256-token blocks, then the blocks ascending)
 *   w_mean[k] = fp32(sum_{j,r} fp32(|W_j[r,k]| / fp32(gmax_j[r, k/gs] + 1e-6f)) / sum_j R_j)
 *       (duo scaling only; gmax = max |W| of the group; same fp64 block order, the
 *        linears' blocks in list order; awq_weight_colsum per linear + awq_column_mean)
 *   candidate i = 0 .. n_grid-1, r = i / n_grid (fp64):
 *       raw_k = max(awq_pow(x_mean_k, r) [/ (awq_pow(w_mean_k, 1-r) + 1e-4)], 1e-4)
 *       s_i[k] = fp32(raw_k / sqrt(max_k raw * min_k raw)), inf / NaN -> 1
 *       (awq_act_scale_table; fp64, IEEE-rounded / and sqrt)
 *   awq_pow(x, r) (round 5; not libm pow, whose last bit differs between math libraries):
 *       r == 0 -> 1; NaN or x < 0 -> NaN; x == 0 -> 0; x == inf -> inf; else, in IEEE fp64
 *       with explicit fma and no other contraction:
 *       ln x: x = m 2^e, m in [sqrt(2)/2, sqrt(2)) (subnormal x scaled by 2^54 first),
 *             f = (m-1)/(m+1); P = 1/25, P = fma(P, f*f, 1/(2j+1)) for j = 11 .. 1;
 *             ln m = fma(2f * (f*f), P, 2f); ln x = fma(e, LN2_HI, fma(e, LN2_LO, ln m))
 *             (LN2_HI = 0x1.62e42feep-1, LN2_LO = 1.90821492927058770002e-10)
 *       e^y:  k = rint(y * 1.44269504088896338700), t = fma(-k, LN2_LO, fma(-k, LN2_HI, y)),
 *             p = 1, p = fma(p, t / j, 1) for j = 15 .. 1; result p * 2^k (k > 1023:
 *             (p 2^1023) 2^(k-1023); k < -1022: (p 2^(k+600)) 2^-600; y > 709.8 -> inf,
 *             y < -746 -> 0)
 *       x^r = e^(r * ln x) — within 2^-40 of x^r over the fp32 range, and the same bits in
 *       every implementation (oracle_act_scale_table restates it)
 *   per element of every group, in the weight dtype D's per-op rounding:
 *       w' = RN_D(w * s_i[k]); RTN scale/zero of w' (awq.py:173-213); q (awq.py:245-248);
 *       dq = fp16(fp16(q - z) * fp16(scale)) (awq.py:459-539); e = fp32(dq / s_i[k]) - w;
 *       c = x_sq[k] * (e * e)
 *   group loss: each 8-element chunk summed in order, then the pairwise tree over the
 *       group's gs/8 chunks (fp32) -> part[i * part_stride + group]
 *       (awq_act_search_losses, per linear at its offset in one group list)
 *   loss_i = fp64 sum in four ascending levels: groups inside a 64-group sub-block,
 *       sub-blocks inside a 1024-group block, blocks inside a 32-block super-block, then
 *       the super-blocks; best = first minimum (NaN never wins; all NaN -> 0)
 *       (awq_act_search_select)
 *   result: every W_j quantized as W_j * diag(s_best) (awq_apply_input_scale, then
 *       awq_quantize_groups); s_best is returned to be folded into the op producing x
 *       (x / s_best, e.g. the preceding norm's weight).
 * The loss is the diagonal (uncorrelated-channel) form of AutoAWQ's output MSE
 * ||x (W' - W)^T||^2.  Weights: bf16 / fp16 / fp32, 2-D, K % gs == 0, gs a power of two in
 * [8, 512]; weights / table / x_sq 16-B aligned.  Sizes of the caller's workspaces:
 *   awq_act_stats      work    fp64 [2 * ceil(T/256) * K]
 *   awq_weight_colsum  gmax_work fp32 [R * K/gs] (scratch of the two-pass path; gs 32 / 64 /
 *                      128 / 256 with 16-B aligned w take the one-pass kernel and leave it
 *                      untouched); partial fp64 [ceil(R/256) * K] (this linear's slice of the
 *                      group's [sum_j ceil(R_j/256), K] array)
 *   awq_act_search_select work fp64 [n_grid * ceil(part_stride / 1024)]
 *   awq_act_scale_table_ws work fp64 [n_grid * (K + 3 * ceil(K / 256))]
 * n_grid <= AWQ_ACT_MAX_GRID; part_stride <= 6144 * 32 * 1024 groups (201 326 592: the
 * select kernel's super-block sums of one candidate fit its LDS), else hipErrorInvalidValue. */
#define AWQ_ACT_MAX_GRID 256

int awq_act_stats(const void* x, int dtype, int64_t tokens, int64_t K, double* work, float* x_mean, float* x_sq,
                  void* stream);
int awq_weight_colsum(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, float* gmax_work,
                      double* partial, void* stream);
/* out[k] = fp32(sum_{b < nblk, ascending} partial[b * K + k] / divisor) (fp64 sum) */
int awq_column_mean(const double* partial, int64_t nblk, int64_t K, double divisor, float* out, void* stream);
/* RTN of W * diag(col_scale) in one pass — the packed outputs of awq_apply_input_scale into a
 * copy followed by awq_quantize_groups on the copy, bit for bit, without the copy (the
 * activation-aware search's last step, round 5).  bf16 / fp16 / fp32 2-D w [rows, K],
 * group_size 32 / 64 / 128 / 256 with K % group_size == 0 and K % 8 == 0, w and col_scale
 * 16-B aligned, packed outputs only (NULL = not wanted); otherwise AWQ_EINVAL (make the two
 * calls).  (ABI 16) */
int awq_quantize_groups_scaled(const void* w, int dtype, int64_t rows, int64_t K, int32_t group_size, int bits,
                               int symmetric, const float* col_scale, int32_t* qweight, int32_t* qzeros,
                               uint16_t* scales, void* stream);
/* table fp32 [n_grid, K]; w_mean NULL = no duo scaling */
int awq_act_scale_table(const float* x_mean, const float* w_mean, int64_t K, int n_grid, float* table,
                        void* stream);
/* The same table (bit for bit) with a caller workspace: every (candidate, channel) power is
 * evaluated once, by one thread, the raw values kept in work between a pass that forms each
 * 256-channel slice's max / min and one that normalises (awq_act_scale_table recomputes the
 * normaliser's pass in each of its workgroups: ~10x the fp64 work, on n_grid x 8 CUs).
 * work fp64 [n_grid * (K + 3 * ceil(K / 256))].  (ABI 16) */
int awq_act_scale_table_ws(const float* x_mean, const float* w_mean, int64_t K, int n_grid, double* work,
                           float* table, void* stream);
/* rtable [n_grid, K] = RN_f32(1 / table) where table is in [2^-60, 2^60], else a NaN (ABI 17;
 * was 0): lets the loss kernel form fp32(dq / s) as one Markstein-corrected product (exact there:
 * awq_selftest 1); a quotient through an out-of-range entry is NaN, and a wave whose candidate
 * loss comes out NaN redoes that candidate with IEEE divisions (the same bits in range). */
int awq_act_recip_table(const float* table, int n_grid, int64_t K, float* rtable, void* stream);
/* rtable: awq_act_recip_table's output for the same table, or NULL (IEEE divisions) */
int awq_act_search_losses(const void* w, int dtype, int64_t rows, int64_t K, int64_t group_size, int bits,
                          int symmetric, const float* table, const float* rtable, int n_grid, const float* x_sq,
                          float* part, int64_t part_stride, void* stream);
/* losses fp64 [n_grid], best int32 [1], s_best fp32 [K] (any may be NULL) */
int awq_act_search_select(const float* part, int n_grid, int64_t part_stride, const float* table, int64_t K,
                          double* work, double* losses, int32_t* best, float* s_best, void* stream);
/* out [rows, K] (dtype D) = RN_D(w * s[k]) */
int awq_apply_input_scale(const void* w, int dtype, int64_t rows, int64_t K, const float* s, void* out,
                          void* stream);

/* Device self-test (diagnostics).  which = 0: the fast reciprocal used by the streaming
 * kernel against IEEE 1/s over every bf16 s >= RN_bf16(1e-10); which = 1: the loss kernel's
 * Markstein quotient against the IEEE division for every s in [1, 2) and every positive
 * finite fp16 dividend; which = 2: the fp16 reciprocal (rcp + one Newton step) against IEEE
 * 1/s over every positive finite fp16 s; adds the number of mismatches to *result (device
 * unsigned long long, caller-zeroed). */
int awq_selftest(int which, unsigned long long* result, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* AWQ_HIP_H */
