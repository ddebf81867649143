/* awq_oracle.h — CPU restatement of the reference quantizer (TEST INFRASTRUCTURE ONLY).
 * See awq_oracle.c for the reference file:line each function follows. */
#ifndef AWQ_ORACLE_H
#define AWQ_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif
enum { AWQ_ORACLE_BF16 = 0, AWQ_ORACLE_F16 = 1, AWQ_ORACLE_F32 = 2, AWQ_ORACLE_F64 = 3 };

/* x: [rows, K] row-major in `dtype`; groups of L along K, tail zero-padded (L >= K: one group).
 * Outputs (any may be NULL): tensor_q int32 [rows, K], scales fp16 bits [rows, G], zeros int32 [rows, G]. */
int oracle_quantize(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym,
                    int32_t* tensor_q, uint16_t* scales_f16, int32_t* zeros);
/* opt-in clip search (product definition, include/awq_hip.h awq_quantize_search) */
int oracle_quantize_search(const void* x, int dtype, int64_t rows, int64_t K, int64_t L, int bits, int sym,
                           int n_grid, int n_cand, int32_t* tensor_q, uint16_t* scales_f16, int32_t* zeros);
int oracle_dequantize(const int32_t* tensor_q, const uint16_t* scales_f16, const int32_t* zeros,
                      int64_t rows, int64_t K, int64_t L, float* out);
int oracle_pack_rows(const int32_t* v, int64_t rows, int64_t n, int bits, int qmin, int32_t* packed);
int oracle_set_threads(int n);
uint16_t oracle_f32_to_bf16(float f);
float oracle_bf16_to_f32(uint16_t h);
uint16_t oracle_f32_to_f16(float f);
float oracle_f16_to_f32(uint16_t h);
#ifdef __cplusplus
}
#endif
#endif
