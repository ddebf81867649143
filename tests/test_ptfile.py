"""Native chunk-file writer (awq_quantizer/ptfile.py + csrc/awq_ptfile.hip): the archive
torch.save writes for the CLI's chunk objects (reference main.py:430-512 saves them with
torch.save), without the GIL.  Checked on CPU: CRC-32 equal to zlib's for every length
class (folded and byte-table paths), files that torch.load (weights_only too) reads back
into the same objects as torch.save's, zip integrity (every record's CRC), fallback to
torch.save for objects outside the supported set, parallel writers."""
import os
import zipfile
import zlib
from concurrent.futures import ThreadPoolExecutor

import pytest
import torch

from awq_quantizer import _hip, ptfile


@pytest.fixture(scope="module")
def lib():
    return _hip.load_library()


@pytest.mark.parametrize("fold", [0, 1])
def test_crc32_matches_zlib(lib, fold):
    rng = torch.Generator().manual_seed(7)
    for n in list(range(0, 200)) + [255, 256, 257, 1023, 4096, 4099, 65536 + 17, (1 << 20) + 3]:
        b = bytes(torch.randint(0, 256, (n,), generator=rng, dtype=torch.uint8).tolist())
        for init in (0, 0xDEADBEEF):
            assert lib.awq_crc32(init, b, n, fold) == zlib.crc32(b, init), (n, init)


def _chunk():
    g = torch.Generator().manual_seed(3)
    d = {}
    for i in range(4):
        d[f"model.layers.{i}.mlp.weight"] = {
            "qweight": torch.randint(-2 ** 31, 2 ** 31 - 1, (64, 16), generator=g, dtype=torch.int32),
            "qzeros": torch.randint(0, 1 << 30, (64, 1), generator=g, dtype=torch.int32),
            "scales": torch.randn(64, 2, generator=g).half(),
            "bits": torch.tensor(4, dtype=torch.int32), "group_size": torch.tensor(128, dtype=torch.int32),
            "symmetric": torch.tensor(False), "shape": torch.tensor([64, 128], dtype=torch.int64),
        }
    d["extra"] = {"bf16": torch.randn(3, 5, generator=g).bfloat16(), "f64": torch.randn(7, generator=g).double(),
                  "u8": torch.arange(9, dtype=torch.uint8).reshape(3, 3), "i8": torch.tensor([-3, 4], dtype=torch.int8),
                  "i16": torch.tensor([[-300]], dtype=torch.int16), "f32": torch.randn(2, 3, 4, 5, generator=g),
                  "empty": torch.empty(0, 7), "big": torch.tensor(2 ** 40), "neg": torch.tensor([-(2 ** 35), -1]),
                  "long_dim": torch.zeros(70000, dtype=torch.int8)}
    d["empty_dict"] = {}
    return d


def _assert_same(a, b):
    assert type(a) is type(b)
    if isinstance(a, dict):
        assert list(a.keys()) == list(b.keys())
        for k in a:
            _assert_same(a[k], b[k])
    else:
        assert a.dtype == b.dtype and a.shape == b.shape and a.stride() == b.stride()
        assert torch.equal(a.view(torch.uint8) if a.dtype == torch.bool else a, b.view(torch.uint8) if b.dtype == torch.bool else b)


@pytest.mark.parametrize("weights_only", [True, False])
def test_same_objects_as_torch_save(tmp_path, weights_only):
    d = _chunk()
    ptfile.save(d, str(tmp_path / "model_chunk_0000.pt"))
    torch.save(d, str(tmp_path / "ref.pt"))
    ours = torch.load(str(tmp_path / "model_chunk_0000.pt"), weights_only=weights_only)
    ref = torch.load(str(tmp_path / "ref.pt"), weights_only=weights_only)
    _assert_same(ours, ref)
    _assert_same(ours, d)


def test_archive_layout_and_crcs(tmp_path):
    p = str(tmp_path / "model_chunk_0003.pt")
    ptfile.save(_chunk(), p)
    torch.save(_chunk(), str(tmp_path / "ref.pt"))
    z, zr = zipfile.ZipFile(p), zipfile.ZipFile(str(tmp_path / "ref.pt"))
    assert z.testzip() is None                                 # every record's CRC-32
    names = [i.filename for i in z.infolist()]
    ref = [i.filename.replace("ref/", "model_chunk_0003/", 1) for i in zr.infolist()]
    assert names == ref                                        # torch.save's records, same order
    for i in z.infolist():
        assert i.compress_type == zipfile.ZIP_STORED
        if "/data/" in i.filename:                             # 64-byte aligned data (mmap loads)
            with open(p, "rb") as f:
                f.seek(i.header_offset + 26)
                nlen, xlen = int.from_bytes(f.read(2), "little"), int.from_bytes(f.read(2), "little")
            assert (i.header_offset + 30 + nlen + xlen) % 64 == 0
    for n in ("version", ".format_version", ".storage_alignment", "byteorder"):
        assert z.read(f"model_chunk_0003/{n}") == zr.read(f"ref/{n}")


def test_unsupported_objects_fall_back(tmp_path):
    for obj in ({"a": [1, 2]}, {"a": {"t": torch.arange(6).reshape(2, 3).t()}}, {1: torch.zeros(2)},
                {"a": torch.zeros(2, requires_grad=True)}):
        p = str(tmp_path / "x.pt")
        ptfile.save(obj, p)
        got = torch.load(p, weights_only=False)
        assert str(got) == str(obj)


def test_parallel_writers(tmp_path):
    d = _chunk()
    paths = [str(tmp_path / f"model_chunk_{i:04d}.pt") for i in range(24)]
    with ThreadPoolExecutor(8) as ex:
        list(ex.map(lambda p: ptfile.save(d, p), paths))
    for p in paths:
        assert zipfile.ZipFile(p).testzip() is None
        _assert_same(torch.load(p, weights_only=True), d)
    assert not os.path.exists(str(tmp_path / "model_chunk_0024.pt"))


def test_too_many_records_falls_back_to_torch_save(tmp_path, lib):
    """The EOCD entry counts are 16-bit: >= 0xFFFF records must go to torch.save (ZIP64)."""
    import ctypes
    n = 0xFFFF
    buf = torch.zeros(n, dtype=torch.int32)
    ptrs = (ctypes.c_void_p * n)(*[buf.data_ptr() + 4 * i for i in range(n)])
    sizes = (ctypes.c_int64 * n)(*([4] * n))
    p = str(tmp_path / "big.pt")
    rc = lib.awq_write_pt(p.encode(), b"big", b"\x80\x02N.", 4, n, ptrs, sizes, b"0" * 40)
    assert rc == 2
    assert not os.path.exists(p)
    # through ptfile.save: the torch.save fallback, which torch.load reads back whole
    d = {f"t{i}": torch.tensor([i], dtype=torch.int32) for i in range(n)}
    ptfile.save(d, p)
    got = torch.load(p, weights_only=True)
    assert len(got) == n and int(got["t65534"][0]) == 65534


def test_save_leaves_python_rng_alone(tmp_path):
    import random
    random.seed(1234)
    want = random.random()
    random.seed(1234)
    ptfile.save(_chunk(), str(tmp_path / "model_chunk_0000.pt"))
    assert random.random() == want


def test_large_archive_parallel_pieces(tmp_path):
    """An archive with > 32 MiB of data is checksummed and written by a thread team in 8 MiB
    pieces at their final offsets (the pieces' CRC-32s combined per record): the file is
    the same archive torch.load reads back, every record's CRC valid."""
    g = torch.Generator().manual_seed(5)
    d = {"big": {"qweight": torch.randint(-2 ** 31, 2 ** 31 - 1, (5000, 2003), generator=g, dtype=torch.int64)
                 .to(torch.int32),                                   # 40 MB: 5 pieces, the last ragged
                 "scales": torch.randn(5000, 17, generator=g).half(), "bits": torch.tensor(4, dtype=torch.int32)},
         "mid": {"tensor_q": torch.randint(0, 16, (3001, 1000), generator=g, dtype=torch.int32)},
         "empty": {"e": torch.empty(0, dtype=torch.int32)}}
    p = str(tmp_path / "model_chunk_0001.pt")
    ptfile.save(d, p)
    z = zipfile.ZipFile(p)
    assert z.testzip() is None
    names = [i.filename for i in z.infolist()]
    torch.save(d, str(tmp_path / "ref.pt"))
    ref = [i.filename.replace("ref/", "model_chunk_0001/", 1) for i in zipfile.ZipFile(str(tmp_path / "ref.pt")).infolist()]
    assert names == ref
    _assert_same(torch.load(p, weights_only=True), d)
    for i in z.infolist():
        if "/data/" in i.filename:
            with open(p, "rb") as f:
                f.seek(i.header_offset + 26)
                nlen, xlen = int.from_bytes(f.read(2), "little"), int.from_bytes(f.read(2), "little")
            assert (i.header_offset + 30 + nlen + xlen) % 64 == 0
