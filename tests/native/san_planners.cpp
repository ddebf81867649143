// ASan/UBSan run of libawq_hip's host-side planning code (no GPU needed): the ragged
// planners (awq_plan_ragged, awq_plan_block_tensor, awq_ragged_flags), the stream pipeline's
// batch planner and argument checks (awq_stream_start: it plans, then fails to create its
// events when no GPU is present), the tuning setter and the quantize entry points' argument
// validation.  TEST INFRASTRUCTURE (tests/native/Makefile, tests/test_sanitizers.py).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/awq_hip.h"

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() { rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17; return rng; }

int main() {
    long checks = 0;
    // ---- ragged planners over random tensor lists ----
    for (int trial = 0; trial < 300; ++trial) {
        const int n = 1 + (int)(next() % 40);
        const int gs = 32 << (next() % 4), bits = (next() & 1) ? 4 : 8;
        std::vector<awq_tensor_desc> d(n);
        for (int i = 0; i < n; ++i) {
            memset(&d[i], 0, sizeof d[i]);
            d[i].w = (const void*)(uintptr_t)(0x100000 + 4096 * i);
            d[i].rows = 1 + (int64_t)(next() % 300);
            int64_t K = gs * (1 + (int64_t)(next() % 20));
            if (next() % 4 == 0) K += 8 * (int64_t)(1 + next() % 3);   // padded rows
            if (next() % 7 == 0) K = 4 + gs * 2;                       // not eligible
            d[i].K = K;
            d[i].qweight = (int32_t*)(uintptr_t)(0x900000 + 64 * i);
            d[i].scales = (uint16_t*)(uintptr_t)(0xA00000 + 64 * i);
        }
        const int64_t total = awq_plan_ragged(d.data(), n, bits, gs);
        ++checks;
        if (total < 0) continue;   // an ineligible tensor: error path
        const int flags = awq_ragged_flags(d.data(), n, gs);
        (void)flags;
        const int64_t need = awq_plan_block_tensor(d.data(), n, total, nullptr, 0);
        std::vector<int32_t> tab((size_t)need + 32);
        int32_t* aligned = (int32_t*)(((uintptr_t)tab.data() + 15) & ~(uintptr_t)15);
        if (awq_plan_block_tensor(d.data(), n, total, aligned, need) != need) { puts("table size"); return 1; }
        if (awq_plan_block_tensor(d.data(), n, total, aligned, need - 1) >= 0) { puts("short table accepted"); return 1; }
        if (awq_plan_block_tensor(d.data(), n, total, aligned + 1, need) >= 0) { puts("misaligned accepted"); return 1; }
        checks += 4;
    }
    // ---- stream pipeline planning (events cannot be created without a GPU: error after planning) ----
    static char host_stage[3 * (65536 + (1 << 20))];   // 3 slots of table area + input
    for (int trial = 0; trial < 200; ++trial) {
        const int n = (int)(next() % 60);
        std::vector<awq_stream_item> it(n);
        for (int i = 0; i < n; ++i) {
            memset(&it[i], 0, sizeof it[i]);
            it[i].fd = 0;
            it[i].dtype = (int)(next() % 4);
            it[i].offset = (int64_t)(next() % 100000);
            it[i].rows = (int64_t)(next() % 700);
            it[i].K = (int64_t)(next() % 900);
            if (next() % 9 == 0) it[i].rows = 0;
            it[i].qweight = (int32_t*)(uintptr_t)0x1000;
        }
        awq_stream_config c;
        memset(&c, 0, sizeof c);
        c.bits = 4; c.symmetric = 0; c.group_size = 128; c.readers = 3; c.nslots = 3;
        c.slot_bytes = 65536; c.first_batch_bytes = (next() & 1) ? 16384 : 0;
        c.host_staging = host_stage; c.dev_staging = (void*)(uintptr_t)0x5000000;
        // the dry-run plan, then random ring gates (valid and invalid) for the start's checks
        std::vector<int32_t> fb((size_t)n + 1), lb((size_t)n + 1);
        const int64_t nb = awq_stream_plan(it.data(), n, &c, fb.data(), lb.data());
        ++checks;
        if (awq_stream_plan(it.data(), n, &c, nullptr, nullptr) != nb) { puts("plan repeat"); return 1; }
        if (nb > 0)
            for (int i = 0; i < n; ++i) {
                if (fb[i] < 0 || lb[i] < fb[i] || lb[i] >= nb) { puts("plan batches"); return 1; }
                if (i > 0 && next() % 4 == 0) it[i].dev_gate = 1 + (int32_t)(next() % (uint64_t)i);
                if (next() % 4 == 0) it[i].host_gate = (int32_t)(next() % (uint64_t)(i + 2));
            }
        void* h = nullptr;
        const int rc = awq_stream_start(it.data(), n, &c, &h);
        if (rc == 0) {   // (a GPU is present after all: run to completion would read fd 0; stop)
            puts("stream started without a GPU");
            return 1;
        }
        ++checks;
    }
    awq_stream_config bad;
    memset(&bad, 0, sizeof bad);
    void* h = nullptr;
    if (awq_stream_start(nullptr, 0, &bad, &h) == 0) { puts("bad config accepted"); return 1; }
    if (awq_stream_table_bytes(1 << 28) <= 0) { puts("table bytes"); return 1; }
    if (awq_stream_release(nullptr, 3) == 0 || awq_stream_plan(nullptr, 2, &bad, nullptr, nullptr) >= 0) {
        puts("null handle / items accepted");
        return 1;
    }
    // ---- argument validation of the launch entry points (no launch reached) ----
    if (awq_quantize_groups_ex(nullptr, 0, 4, 256, 128, 3, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == 0 ||
        awq_quantize_groups_ex(nullptr, 0, 4, 256, 0, 4, 0, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == 0 ||
        awq_quantize_groups_ex(nullptr, 0, 4, 256, 128, 4, 0, 7, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr) == 0 ||
        awq_quantize_search_ex(nullptr, 0, 4, 256, 128, 4, 0, 0, 5, 9, nullptr, nullptr, nullptr, nullptr, nullptr,
                               nullptr) == 0) {
        puts("bad launch arguments accepted");
        return 1;
    }
    checks += 8;
    printf("san_planners: %ld checks clean (last error: %s)\n", checks, awq_last_error());
    return 0;
}
