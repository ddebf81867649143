/*
 * awq_ptfile.h — native writer of the CLI's chunk files (libawq_hip.so, host code only).
 *
 * NOT a replacement of a reference compute interface: the reference saves its chunk objects
 * with torch.save (src/awq_quantizer/main.py:430-512, save_model_in_chunks).  This writes
 * the same archive (record names and order, stored 64-byte aligned records, data
 * descriptors, CRC-32) from pickle bytes and tensor buffers built by the caller
 * (awq_quantizer/ptfile.py), so that chunk files are written without the Python GIL.
 */
#ifndef AWQ_PTFILE_H
#define AWQ_PTFILE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* CRC-32 as zlib's crc32(crc, data, n); fold = 0 forces the byte-table path. */
uint32_t awq_crc32(uint32_t crc, const void* data, int64_t n, int32_t fold);

/* Archive <archive>/{data.pkl, .format_version, .storage_alignment, byteorder, data/0..n-1,
 * version, .data/serialization_id} at path.  Returns 0 written, 1 I/O error, 2 needs ZIP64
 * (>= 2^32 - 1 bytes: use torch.save), 3 bad arguments. */
int awq_write_pt(const char* path, const char* archive, const char* pkl, int64_t pkl_len, int32_t n,
                 const void* const* ptrs, const int64_t* sizes, const char* serialization_id);

#ifdef __cplusplus
}
#endif
#endif /* AWQ_PTFILE_H */
