"""Host-side planning of the native pipeline's bounded output memory (awq_quantizer/stream.py,
include/awq_hip.h awq_stream_plan / dev_gate / host_gate), CPU only: ring placement, the
batch plan the gates are validated against, the ring sizing, and the library's rejection of
a gate that could deadlock.  (The pipeline itself runs in tests/test_cli.py, -m gpu.)"""
import ctypes
import random

import pytest

from awq_quantizer import _hip
from awq_quantizer import stream as S


def _overlap(a, b):
    return a[0] < b[1] and b[0] < a[1]


@pytest.mark.parametrize("seed", range(20))
def test_ring_place_gates_are_the_latest_overwritten_region(seed):
    rng = random.Random(seed)
    sizes = [rng.choice([1, 2, 3, 7, 16]) * S.ALIGN for _ in range(rng.randint(1, 60))]
    cap = rng.choice([16, 20, 33, 64]) * S.ALIGN
    p = S.ring_place(sizes, cap)
    if max(sizes) > cap:
        assert p is None
        return
    offs, gates = p
    for i, (o, sz) in enumerate(zip(offs, sizes)):
        assert 0 <= o and o + sz <= cap
        # brute force: the latest earlier region still holding bytes this one overwrites
        want = 0
        for j in range(i):
            # region j is still intact at time i unless a region between j and i overwrote it
            span = (offs[j], offs[j] + sizes[j])
            dead = any(_overlap(span, (offs[k], offs[k] + sizes[k])) for k in range(j + 1, i))
            if not dead and _overlap(span, (o, o + sz)):
                want = j + 1
        assert gates[i] == want
        assert gates[i] <= i
        if gates[i]:
            j = gates[i] - 1
            assert _overlap((offs[j], offs[j] + sizes[j]), (o, o + sz))


def test_ring_place_no_wrap_when_everything_fits():
    offs, gates = S.ring_place([S.ALIGN] * 10, 10 * S.ALIGN)
    assert offs == [k * S.ALIGN for k in range(10)] and gates == [0] * 10


def test_region_layout_fields_aligned():
    f, size = S.region_layout((1000, 300), 1000, 300, 100, 4, True)
    assert [x[0] for x in f] == ["qweight", "qzeros", "scales"]
    assert all(off % S.ALIGN == 0 for _, _, _, off, _ in f)
    assert f[0][4] == 1000 * 38 * 4 and f[1][4] == 1000 * 1 * 4 and f[2][4] == 1000 * 3 * 2
    assert size % S.ALIGN == 0 and size >= f[-1][3] + f[-1][4]
    f, _ = S.region_layout((8, 3, 128), 8, 384, 128, 4, False)
    assert [x[0] for x in f] == ["tensor_q", "scales", "zero_points"] and f[0][1] == (8, 3, 128)


def _items(shapes):
    arr = (_hip.StreamItem * len(shapes))()
    for k, (rows, K) in enumerate(shapes):
        arr[k].fd, arr[k].dtype, arr[k].rows, arr[k].K = 0, 0, rows, K
    return arr


def _plan(shapes, slot, first_bytes=0):
    lib = _hip.load_library()
    arr = _items(shapes)
    cfg = _hip.StreamConfig(bits=4, group_size=128, readers=1, nslots=3, slot_bytes=slot,
                            first_batch_bytes=first_bytes)
    n = len(shapes)
    fb, lb = (ctypes.c_int32 * n)(), (ctypes.c_int32 * n)()
    nb = lib.awq_stream_plan(arr, n, ctypes.byref(cfg), fb, lb)
    return nb, list(fb), list(lb)


def test_stream_plan_batches():
    # 4 KiB slots: 2 rows of 1024 bf16 per slot; a 5-row tensor spans 3 batches
    nb, fb, lb = _plan([(1, 1024), (5, 1024), (1, 1024), (1, 512), (1, 512)], 4096)
    assert nb > 0
    assert fb[0] == lb[0] == 0
    assert fb[1] <= lb[1] and lb[1] - fb[1] >= 2
    assert all(lb[i] <= lb[i + 1] for i in range(4)) and all(fb[i] <= lb[i] for i in range(5))
    assert lb[-1] == nb - 1


def test_stream_plan_rejects_a_row_larger_than_the_slot():
    nb, _, _ = _plan([(2, 4096)], 4096)
    assert nb < 0 and "does not fit" in _hip.last_error()


def _sizes_plan(rng):
    shapes = [(rng.choice([1, 3, 8, 40]), rng.choice([256, 1024, 2048])) for _ in range(rng.randint(5, 80))]
    nb, fb, lb = _plan(shapes, 8192)
    assert nb > 0
    sizes = [S.region_layout((r, K), r, K, 128, 4, True)[1] for r, K in shapes]
    return shapes, sizes, fb, lb


@pytest.mark.parametrize("seed", range(10))
def test_size_ring_satisfies_both_gate_rules(seed):
    rng = random.Random(seed)
    _, sizes, fb, lb = _sizes_plan(rng)
    n = len(sizes)
    group = [k // rng.choice([1, 2, 4, 10]) for k in range(n)]
    gend = [max(j for j in range(n) if group[j] == group[k]) for k in range(n)]
    cap, offs, gates = S.size_ring(sizes, 4 * S.ALIGN, lambda g: S.dev_gates_ok(g, fb, lb))
    assert S.dev_gates_ok(gates, fb, lb)
    assert cap >= max(sizes)
    cap, offs, gates = S.size_ring(sizes, 4 * S.ALIGN, lambda g: S.host_gates_ok(g, lb, gend))
    assert S.host_gates_ok(gates, lb, gend)
    # a deliberately tiny ring that wraps inside one batch is refused by the rule
    p = S.ring_place(sizes, max(sizes))
    if any(p[1]) and any(g and lb[g - 1] >= fb[i] for i, g in enumerate(p[1])):
        assert not S.dev_gates_ok(p[1], fb, lb)


def test_start_rejects_a_device_gate_that_waits_on_its_own_batch():
    """awq_stream_start validates the gates against its plan before touching the GPU."""
    lib = _hip.load_library()
    arr = _items([(1, 1024), (1, 1024)])
    for k in range(2):
        arr[k].qweight = 4096 * (k + 1)
    arr[1].dev_gate = 1                      # both items land in one batch: would deadlock
    cfg = _hip.StreamConfig(bits=4, group_size=128, readers=1, nslots=3, slot_bytes=1 << 20,
                            host_staging=4096, dev_staging=4096)
    h = ctypes.c_void_p()
    rc = lib.awq_stream_start(arr, 2, ctypes.byref(cfg), ctypes.byref(h))
    assert rc == 1 and "device output ring too small" in _hip.last_error()
    arr[1].dev_gate = 2                      # an item cannot wait for itself
    rc = lib.awq_stream_start(arr, 2, ctypes.byref(cfg), ctypes.byref(h))
    assert rc == 1 and "earlier items" in _hip.last_error()
    cfg.search_grid, cfg.search_candidates = 4, 5
    arr[1].dev_gate = 0
    rc = lib.awq_stream_start(arr, 2, ctypes.byref(cfg), ctypes.byref(h))
    assert rc == 1 and "search" in _hip.last_error()


def test_writer_groups_and_hooks(tmp_path):
    import torch
    from awq_quantizer.main import ChunkWriter
    names = [f"t{k}" for k in range(7)]
    w = ChunkWriter(names, str(tmp_path), 3, False)
    got = []
    w.add_written_hook(lambda ns: got.append(list(ns)))
    w.done("t1", None)
    assert w.predict_groups() == {"t0": 0, "t2": 0, "t3": 0, "t4": 1, "t5": 1, "t6": 1}
    r = {"qweight": torch.zeros(2, 2, dtype=torch.int32)}
    for n in names:
        if n != "t1":
            w.done(n, dict(r))
    w.close()
    assert sorted(map(tuple, got)) == [("t0", "t2", "t3"), ("t4", "t5", "t6")]
