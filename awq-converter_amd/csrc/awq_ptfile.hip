// awq_ptfile.hip — the CLI's chunk files (model_chunk_NNNN.pt, reference main.py:430-512)
// written natively, host code only.
//
// torch.save holds the Python GIL through its pickler and through the zip writer's CRC-32
// and copies (measured in the build container: 0.67 GB/s for a 5.4 MB packed chunk with 1,
// 2, 4 or 8 writer threads alike), which made the chunk files the CLI's critical path
// once the GPU pipeline went native.  Here the caller (main.py, awq_quantizer/ptfile.py)
// hands over the pickle bytes it built and the tensors' host pointers; this writes the
// archive torch.save writes — the same record names and order, stored (uncompressed)
// records whose data start on 64-byte boundaries (an "FB" padding extra field), a data
// descriptor after every record, a central directory — with the standard CRC-32 of every
// record (PCLMULQDQ folding, byte table for the tail), without the GIL (ctypes releases
// it), so chunk files are written in parallel.  torch.load (weights_only=True too) reads
// them back into the same objects.  Archives whose offsets or sizes would need ZIP64
// (>= 2^32 - 1 bytes) are refused (return 2): the caller falls back to torch.save.
#include "../../include/awq_ptfile.h"

#include <fcntl.h>
#include <immintrin.h>
#include <sys/uio.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

struct CrcTable {
    uint32_t t[256];
    CrcTable() {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t c = i;
            for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            t[i] = c;
        }
    }
};
const CrcTable kCrc;

uint32_t crc_bytes(uint32_t c, const unsigned char* p, size_t n) {   // c: the inverted register
    for (size_t i = 0; i < n; ++i) c = kCrc.t[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c;
}

// one 128-bit fold: acc * x^128 (mod P) split over the two 64-bit halves, + next
__attribute__((target("pclmul,sse4.1"))) inline __m128i fold16(__m128i acc, __m128i next, __m128i k) {
    const __m128i lo = _mm_clmulepi64_si128(acc, k, 0x00);
    return _mm_xor_si128(_mm_xor_si128(_mm_clmulepi64_si128(acc, k, 0x11), next), lo);
}

// CRC-32 (reflected 0x04C11DB7) of n >= 64 bytes, n % 16 == 0, by carry-less multiply
// folding (Gopal et al., "Fast CRC Computation for Generic Polynomials Using PCLMULQDQ"):
// four 128-bit lanes folded by 512 bits per step, merged, folded by 128 bits, reduced to
// 64 and then (Barrett) to 32 bits.  c: the inverted register in and out.
__attribute__((target("pclmul,sse4.1"))) uint32_t crc_fold(uint32_t c, const unsigned char* p, size_t n) {
    alignas(16) static const uint64_t k1k2[2] = {0x0154442bd4ull, 0x01c6e41596ull};
    alignas(16) static const uint64_t k3k4[2] = {0x01751997d0ull, 0x00ccaa009eull};
    alignas(16) static const uint64_t k5k0[2] = {0x0163cd6124ull, 0x0ull};
    alignas(16) static const uint64_t poly[2] = {0x01db710641ull, 0x01f7011641ull};
    __m128i x1 = _mm_loadu_si128((const __m128i*)(p + 0));
    __m128i x2 = _mm_loadu_si128((const __m128i*)(p + 16));
    __m128i x3 = _mm_loadu_si128((const __m128i*)(p + 32));
    __m128i x4 = _mm_loadu_si128((const __m128i*)(p + 48));
    x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)c));
    __m128i k = _mm_load_si128((const __m128i*)k1k2);
    p += 64;
    n -= 64;
    while (n >= 64) {
        const __m128i a1 = _mm_clmulepi64_si128(x1, k, 0x00), a2 = _mm_clmulepi64_si128(x2, k, 0x00);
        const __m128i a3 = _mm_clmulepi64_si128(x3, k, 0x00), a4 = _mm_clmulepi64_si128(x4, k, 0x00);
        x1 = _mm_clmulepi64_si128(x1, k, 0x11);
        x2 = _mm_clmulepi64_si128(x2, k, 0x11);
        x3 = _mm_clmulepi64_si128(x3, k, 0x11);
        x4 = _mm_clmulepi64_si128(x4, k, 0x11);
        x1 = _mm_xor_si128(_mm_xor_si128(x1, a1), _mm_loadu_si128((const __m128i*)(p + 0)));
        x2 = _mm_xor_si128(_mm_xor_si128(x2, a2), _mm_loadu_si128((const __m128i*)(p + 16)));
        x3 = _mm_xor_si128(_mm_xor_si128(x3, a3), _mm_loadu_si128((const __m128i*)(p + 32)));
        x4 = _mm_xor_si128(_mm_xor_si128(x4, a4), _mm_loadu_si128((const __m128i*)(p + 48)));
        p += 64;
        n -= 64;
    }
    k = _mm_load_si128((const __m128i*)k3k4);
    x1 = fold16(x1, x2, k);
    x1 = fold16(x1, x3, k);
    x1 = fold16(x1, x4, k);
    while (n >= 16) {
        x1 = fold16(x1, _mm_loadu_si128((const __m128i*)p), k);
        p += 16;
        n -= 16;
    }
    // 128 -> 64 bits
    const __m128i mask32 = _mm_setr_epi32(~0, 0, ~0, 0);
    x2 = _mm_clmulepi64_si128(x1, k, 0x10);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2);
    k = _mm_loadl_epi64((const __m128i*)k5k0);
    x2 = _mm_srli_si128(x1, 4);
    x1 = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k, 0x00), x2);
    // Barrett reduction to 32 bits
    k = _mm_load_si128((const __m128i*)poly);
    x2 = _mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k, 0x10);
    x2 = _mm_clmulepi64_si128(_mm_and_si128(x2, mask32), k, 0x00);
    x1 = _mm_xor_si128(x1, x2);
    return (uint32_t)_mm_extract_epi32(x1, 1);
}

bool have_clmul() {
    static const bool ok = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
    return ok;
}

uint32_t crc32_of(uint32_t crc, const void* data, size_t n, bool fold) {
    const unsigned char* p = (const unsigned char*)data;
    uint32_t c = ~crc;
    if (fold && n >= 64) {
        const size_t m = n & ~(size_t)15;
        c = crc_fold(c, p, m);
        p += m;
        n -= m;
    }
    return ~crc_bytes(c, p, n);
}

void put16(std::string& s, uint32_t v) {
    s.push_back((char)(v & 0xFF));
    s.push_back((char)((v >> 8) & 0xFF));
}
void put32(std::string& s, uint32_t v) {
    put16(s, v & 0xFFFF);
    put16(s, v >> 16);
}

bool write_all(int fd, std::vector<iovec>& iov) {
    size_t i = 0;
    while (i < iov.size()) {
        const int cnt = (int)std::min<size_t>(iov.size() - i, 512);
        const ssize_t w = writev(fd, &iov[i], cnt);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        size_t left = (size_t)w;
        while (left > 0 && i < iov.size()) {
            if (left >= iov[i].iov_len) {
                left -= iov[i].iov_len;
                ++i;
            } else {
                iov[i].iov_base = (char*)iov[i].iov_base + left;
                iov[i].iov_len -= left;
                left = 0;
            }
        }
        while (i < iov.size() && iov[i].iov_len == 0) ++i;
    }
    return true;
}

// CRC-32 of A || B from crc(A), crc(B) and len(B): zlib's crc32_combine (the GF(2) operator
// that appends len(B) zero bytes, by repeated squaring), so a record's pieces can be
// checksummed by different threads
uint32_t gf2_times(const uint32_t* mat, uint32_t vec) {
    uint32_t sum = 0;
    for (; vec; vec >>= 1, ++mat)
        if (vec & 1) sum ^= *mat;
    return sum;
}
void gf2_square(uint32_t* sq, const uint32_t* mat) {
    for (int n = 0; n < 32; ++n) sq[n] = gf2_times(mat, mat[n]);
}
uint32_t crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
    if (len2 == 0) return crc1;
    uint32_t even[32], odd[32];
    odd[0] = 0xEDB88320u;   // the operator for one zero bit
    for (uint32_t n = 1, row = 1; n < 32; ++n, row <<= 1) odd[n] = row;
    gf2_square(even, odd);   // two zero bits
    gf2_square(odd, even);   // four
    do {
        gf2_square(even, odd);
        if (len2 & 1) crc1 = gf2_times(even, crc1);
        len2 >>= 1;
        if (!len2) break;
        gf2_square(odd, even);
        if (len2 & 1) crc1 = gf2_times(odd, crc1);
        len2 >>= 1;
    } while (len2);
    return crc1 ^ crc2;
}

bool pwrite_all(int fd, const void* data, size_t n, uint64_t off) {
    const char* p = (const char*)data;
    while (n > 0) {
        const ssize_t w = pwrite(fd, p, n, (off_t)off);
        if (w < 0) {
            if (errno == EINTR) continue;
            return false;
        }
        p += w;
        n -= (size_t)w;
        off += (uint64_t)w;
    }
    return true;
}

constexpr uint64_t kPiece = 8ull << 20;            // checksum + write unit of a large archive
constexpr uint64_t kParallelBytes = 32ull << 20;   // archives with more data go to a thread team

}  // namespace

extern "C" {

// CRC-32 (zlib's crc32(crc, data, n)); fold = 0 forces the byte table (tests)
uint32_t awq_crc32(uint32_t crc, const void* data, int64_t n, int32_t fold) {
    return crc32_of(crc, data, (size_t)n, fold != 0 && have_clmul());
}

// torch.save's archive for one object: records <archive>/data.pkl (pkl), .format_version,
// .storage_alignment, byteorder, data/0 .. data/<n - 1> (ptrs[i], sizes[i] bytes), version,
// .data/serialization_id (40 characters).  0 = written, 1 = I/O error (errno kept),
// 2 = needs ZIP64 (caller falls back), 3 = bad arguments.
int awq_write_pt(const char* path, const char* archive, const char* pkl, int64_t pkl_len, int32_t n,
                 const void* const* ptrs, const int64_t* sizes, const char* serialization_id) {
    if (!path || !archive || !pkl || pkl_len < 0 || n < 0 || (n > 0 && (!ptrs || !sizes)) || !serialization_id ||
        strlen(serialization_id) != 40)
        return 3;
    struct Rec {
        std::string name;
        const void* data;
        uint64_t size;
        uint32_t crc;
        uint64_t offset;
    };
    const std::string a(archive);
    std::vector<Rec> recs;
    recs.reserve((size_t)n + 7);
    recs.push_back({a + "/data.pkl", pkl, (uint64_t)pkl_len, 0, 0});
    recs.push_back({a + "/.format_version", "1", 1, 0, 0});
    recs.push_back({a + "/.storage_alignment", "64", 2, 0, 0});
    recs.push_back({a + "/byteorder", "little", 6, 0, 0});
    for (int32_t i = 0; i < n; ++i) {
        if (sizes[i] < 0 || (sizes[i] > 0 && !ptrs[i])) return 3;
        recs.push_back({a + "/data/" + std::to_string(i), ptrs[i], (uint64_t)sizes[i], 0, 0});
    }
    recs.push_back({a + "/version", "3\n", 2, 0, 0});
    recs.push_back({a + "/.data/serialization_id", serialization_id, 40, 0, 0});
    const bool fold = have_clmul();
    // layout and headers (local header + FB padding so the data start on 64 B); the data
    // descriptors carry the CRCs and follow once they are known
    std::vector<std::string> heads(recs.size());
    static const char kPad[64] = {'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z',
                                  'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z',
                                  'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z',
                                  'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z', 'Z'};
    std::vector<std::string> descs(recs.size());
    std::vector<uint64_t> data_off(recs.size());
    uint64_t off = 0, total_data = 0;
    const uint64_t kLim = 0xFFFFFFFFull;
    constexpr uint64_t kDesc = 16;                 // data descriptor: signature, crc, 2 sizes
    for (size_t i = 0; i < recs.size(); ++i) {
        Rec& r = recs[i];
        if (r.size >= kLim) return 2;
        r.offset = off;
        const uint64_t pre = 30 + r.name.size() + 4;
        const uint32_t pad = (uint32_t)((64 - (off + pre) % 64) % 64);
        std::string& h = heads[i];
        put32(h, 0x04034b50u);
        put16(h, 0);              // version needed
        put16(h, 0x0808);         // data descriptor follows, UTF-8 names
        put16(h, 0);              // stored
        put16(h, 0);              // time
        put16(h, 0);              // date
        put32(h, 0);              // crc, sizes: in the data descriptor
        put32(h, 0);
        put32(h, 0);
        put16(h, (uint32_t)r.name.size());
        put16(h, 4 + pad);
        h += r.name;
        h += "FB";
        put16(h, pad);
        h.append(kPad, pad);
        data_off[i] = off + h.size();
        off += h.size() + r.size + kDesc;
        total_data += r.size;
        if (off >= kLim) return 2;
    }
    // the EOCD's entry counts are 16-bit: a larger archive needs ZIP64 (torch.save writes it)
    if (recs.size() >= 0xFFFF) return 2;
    const int fd = open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
    if (fd < 0) return 1;
    // CRCs (and, for a large archive, the data itself): a large archive's records are cut
    // into 8 MiB pieces that a team of threads checksums and writes at their final offsets
    // (pwrite), the pieces' CRCs combined per record — one chunk of a few GB (the reference
    // format's int32 tensor_q) no longer serialises on one thread (round 4: it stalled the
    // CLI pipeline's host-ring reuse)
    const bool parallel = total_data >= kParallelBytes;
    bool io_ok = true;
    int io_errno = 0;
    if (parallel) {
        struct Piece {
            size_t rec;
            uint64_t at, len;
            uint32_t crc;
        };
        std::vector<Piece> pieces;
        for (size_t i = 0; i < recs.size(); ++i)
            for (uint64_t a = 0; a < recs[i].size; a += kPiece)
                pieces.push_back({i, a, std::min(kPiece, recs[i].size - a), 0u});
        const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
        const int team = (int)std::min<uint64_t>({8ull, (uint64_t)hw, (total_data + kParallelBytes - 1) / kParallelBytes * 2,
                                                  (uint64_t)pieces.size()});
        std::atomic<size_t> next{0};
        std::atomic<bool> failed{false};
        std::atomic<int> err{0};
        auto work = [&]() {
            for (size_t k; (k = next.fetch_add(1)) < pieces.size() && !failed.load();) {
                Piece& pc = pieces[k];
                const unsigned char* src = (const unsigned char*)recs[pc.rec].data + pc.at;
                pc.crc = crc32_of(0, src, (size_t)pc.len, fold);
                if (!pwrite_all(fd, src, (size_t)pc.len, data_off[pc.rec] + pc.at)) {
                    err.store(errno);
                    failed.store(true);
                }
            }
        };
        std::vector<std::thread> th;
        for (int t = 1; t < team; ++t) th.emplace_back(work);
        work();
        for (auto& t : th) t.join();
        io_ok = !failed.load();
        io_errno = err.load();
        for (Rec& r : recs) r.crc = 0;
        for (const Piece& pc : pieces) recs[pc.rec].crc = crc32_combine(recs[pc.rec].crc, pc.crc, pc.len);
    } else {
        for (Rec& r : recs) r.crc = r.size ? crc32_of(0, r.data, (size_t)r.size, fold) : 0u;
    }
    for (size_t i = 0; i < recs.size(); ++i) {
        std::string& d = descs[i];
        put32(d, 0x08074b50u);
        put32(d, recs[i].crc);
        put32(d, (uint32_t)recs[i].size);
        put32(d, (uint32_t)recs[i].size);
    }
    std::string cd;
    for (const Rec& r : recs) {
        put32(cd, 0x02014b50u);
        put16(cd, 0);             // version made by
        put16(cd, 0);             // version needed
        put16(cd, 0x0808);
        put16(cd, 0);
        put16(cd, 0);
        put16(cd, 0);
        put32(cd, r.crc);
        put32(cd, (uint32_t)r.size);
        put32(cd, (uint32_t)r.size);
        put16(cd, (uint32_t)r.name.size());
        put16(cd, 0);             // extra
        put16(cd, 0);             // comment
        put16(cd, 0);             // disk
        put16(cd, 0);             // internal attributes
        put32(cd, 0);             // external attributes
        put32(cd, (uint32_t)r.offset);
        cd += r.name;
    }
    if (off + cd.size() + 22 >= kLim) {
        close(fd);
        unlink(path);
        return 2;
    }
    std::string eocd;
    put32(eocd, 0x06054b50u);
    put16(eocd, 0);
    put16(eocd, 0);
    put16(eocd, (uint32_t)recs.size());
    put16(eocd, (uint32_t)recs.size());
    put32(eocd, (uint32_t)cd.size());
    put32(eocd, (uint32_t)off);
    put16(eocd, 0);
    if (io_ok && parallel) {
        // the data are in place: headers, descriptors, central directory, EOCD at their offsets
        for (size_t i = 0; i < recs.size() && io_ok; ++i)
            io_ok = pwrite_all(fd, heads[i].data(), heads[i].size(), recs[i].offset) &&
                    pwrite_all(fd, descs[i].data(), descs[i].size(), data_off[i] + recs[i].size);
        io_ok = io_ok && pwrite_all(fd, cd.data(), cd.size(), off) &&
                pwrite_all(fd, eocd.data(), eocd.size(), off + cd.size());
        if (!io_ok) io_errno = errno;
    } else if (io_ok) {
        std::vector<iovec> iov;
        iov.reserve(recs.size() * 3 + 2);
        for (size_t i = 0; i < recs.size(); ++i) {
            iov.push_back({(void*)heads[i].data(), heads[i].size()});
            if (recs[i].size) iov.push_back({const_cast<void*>(recs[i].data), (size_t)recs[i].size});
            iov.push_back({(void*)descs[i].data(), descs[i].size()});
        }
        iov.push_back({(void*)cd.data(), cd.size()});
        iov.push_back({(void*)eocd.data(), eocd.size()});
        io_ok = write_all(fd, iov);
        if (!io_ok) io_errno = errno;
    }
    if (close(fd) != 0 || !io_ok) {
        errno = io_ok ? errno : io_errno;
        return 1;
    }
    return 0;
}

}  // extern "C"
