"""CPU tests of the host-only parts of the weight / solver-state files
 and of the genetic strategy's generator (§8f-4).

Pinning: the binary fixtures in tests/golden/ were serialised by protobuf
itself over the reference's caffe.proto (tests/golden/make_proto_golden.py);
the generator is checked against this machine's glibc rand()."""
import ctypes
import json
import struct
from pathlib import Path

import pytest

GOLD = Path(__file__).resolve().parent / "golden"


def _rows(desc):
    return [[n, t, i, list(s), c, d, nd] for (n, t, i, s, c, d, nd) in desc]


def test_caffemodel_v2_parse_matches_protobuf_fixture():
    from rramsim import caffe
    exp = json.loads((GOLD / "proto_golden.json").read_text())["tiny_net"]
    got = _rows(caffe.caffemodel_describe(GOLD / "tiny_net.caffemodel"))
    assert [r[:5] + [r[6]] for r in got] == [r[:5] + [r[6]] for r in exp]
    for g, e in zip(got, exp):
        assert g[5] == pytest.approx(e[5], abs=1e-6)


def test_caffemodel_v1_layers_with_legacy_dims():
    from rramsim import caffe
    exp = json.loads((GOLD / "proto_golden.json").read_text())["tiny_v1"]
    got = _rows(caffe.caffemodel_describe(GOLD / "tiny_v1.caffemodel"))
    assert [r[:5] for r in got] == [r[:5] for r in exp]


def test_net_serialiser_is_byte_identical_to_protobuf(tmp_path):
    """Our writer emits the fields protobuf's serializer would, in the same order."""
    from rramsim import caffe
    out = tmp_path / "re.caffemodel"
    caffe.proto_rewrite(GOLD / "tiny_net.caffemodel", out, "net")
    assert out.read_bytes() == (GOLD / "tiny_net.caffemodel").read_bytes()


def test_solverstate_round_trip_is_byte_identical(tmp_path):
    from rramsim import caffe
    out = tmp_path / "re.solverstate"
    caffe.proto_rewrite(GOLD / "tiny.solverstate", out, "solverstate")
    assert out.read_bytes() == (GOLD / "tiny.solverstate").read_bytes()


def test_v1_model_upgrades_to_layer_format(tmp_path):
    from rramsim import caffe
    out = tmp_path / "v2.caffemodel"
    caffe.proto_rewrite(GOLD / "tiny_v1.caffemodel", out, "net")
    a = caffe.caffemodel_describe(GOLD / "tiny_v1.caffemodel")
    b = caffe.caffemodel_describe(out)
    assert a == b
    assert b"\xa2\x06" in out.read_bytes()  # field 100 (`layer`), length-delimited


def test_malformed_proto_fails_cleanly(tmp_path):
    from rramsim import caffe
    from rramsim._kernels import RramError
    bad = tmp_path / "bad.caffemodel"
    bad.write_bytes(b"\xa2\x06\xff\xff\x03")  # layer with a length past the end
    with pytest.raises(RramError, match="overruns"):
        caffe.caffemodel_describe(bad)
    with pytest.raises(RramError, match="cannot open"):
        caffe.caffemodel_describe(tmp_path / "missing.caffemodel")


def test_packed_and_unpacked_floats_both_parse(tmp_path):
    """protobuf accepts both encodings of a repeated float; so must we."""
    from rramsim import caffe

    def varint(v):
        out = b""
        while v >= 0x80:
            out += bytes([(v & 0x7F) | 0x80])
            v >>= 7
        return out + bytes([v])

    def ld(field, payload):
        return varint(field << 3 | 2) + varint(len(payload)) + payload
    unpacked = b"".join(varint(5 << 3 | 5) + struct.pack("<f", x) for x in (1.0, 2.0, 3.5))
    shape = ld(7, ld(1, varint(3)))
    blob = unpacked + shape
    layer = ld(1, b"L") + ld(2, b"InnerProduct") + ld(7, blob)
    f = tmp_path / "u.caffemodel"
    f.write_bytes(ld(100, layer))
    (name, typ, idx, shp, n, s, nd), = caffe.caffemodel_describe(f)
    assert (name, typ, idx, shp, n, s, nd) == ("L", "InnerProduct", 0, (3,), 3, 6.5, 0)


@pytest.mark.parametrize("seed", [1, 0, 42, 1701, 2**31 - 1])
def test_glibc_rand_matches_libc(seed):
    """GeneticFailureStrategy's unseeded rand() (strategy.cpp:170-175) is glibc's
    TYPE_3 generator at seed 1; check ours against this machine's libc."""
    from rramsim import caffe
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(ctypes.c_uint(seed))
    want = [libc.rand() for _ in range(2000)]
    assert caffe.glibc_rand(seed, 2000) == want
