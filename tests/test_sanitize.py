"""ASan + UBSan run of the host parsers (SURVEY.md §5 "Run the host build under
ASan/UBSan in CPU tests").

`make -C rram-caffe-simulation_amd sanitize` compiles the product's own
host/proto.cpp (text prototxt) and host/io.cpp (binary .caffemodel /
.solverstate / blob-vector codec) with -fsanitize=address,undefined (+
float-cast-overflow, no recovery) into tests/sanitize/parse_fuzz.cpp's driver.
Each input must parse and round-trip; thousands of truncated / bit-flipped /
spliced / oversized-length / deeply nested copies must each either parse or
fail with the error the C-ABI reports as RRAM_EINVAL, with zero sanitizer
reports.  The malformed files are also fed through the shipped library's
C-ABI (no sanitizer) to show the status code, not a crash, comes back.
"""
import ctypes
import os
import shutil
import struct
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "rram-caffe-simulation_amd"
DRIVER = PKG / "build_asan" / "parse_fuzz"
GOLD = ROOT / "tests" / "golden"
REF = Path("/root/reference")


@pytest.fixture(scope="module")
def driver():
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    subprocess.run(["make", "-s", "-C", str(PKG), "sanitize"], check=True)
    return DRIVER


def _run(driver, kind, path, n=3000, seed=1701):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([str(driver), kind, str(path), str(n), str(seed)], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, f"{kind} {path}: rc={r.returncode}\n{r.stdout}\n{r.stderr[-4000:]}"
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert "0 crashes" in r.stdout
    return r.stdout


def _blob(data, shape):
    """BlobProto wire bytes: packed data (field 5) + BlobShape (field 7)."""
    def varint(v):
        out = b""
        while v >= 0x80:
            out += bytes([(v & 0x7F) | 0x80])
            v >>= 7
        return out + bytes([v])
    dims = b"".join(varint(d) for d in shape)
    shp = b"\x0a" + varint(len(dims)) + dims
    payload = struct.pack(f"<{len(data)}f", *data)
    return b"\x2a" + varint(len(payload)) + payload + b"\x3a" + varint(len(shp)) + shp


def test_binary_formats_under_asan_ubsan(driver, tmp_path):
    outs = [_run(driver, "net", GOLD / "tiny_net.caffemodel"),
            _run(driver, "net", GOLD / "tiny_v1.caffemodel"),
            _run(driver, "solverstate", GOLD / "tiny.solverstate")]
    fs = tmp_path / "x.faultstate"                      # .faultstate = BlobProtoVector (Q11 extension)
    blobs = [_blob([1.0, -2.5, 3.0e6, 0.0], [2, 2]), _blob([-1.0, 0.0, 1.0], [3]), _blob([], [0])]
    fs.write_bytes(b"".join(b"\x0a" + bytes([len(b)]) + b for b in blobs))
    outs.append(_run(driver, "blobs", fs))
    for o in outs:
        assert "RRAM_EINVAL" in o


def test_prototxts_under_asan_ubsan(driver, tmp_path):
    from rramsim import models
    texts = {name: f() for name, (f, _, _) in models.CONFIGS.items()}
    texts["solver"] = models.solver(failure_mean=5e6, failure_std=1.5e6, failure_prob=(5, 90, 5), threshold=1e-3)
    paths = []
    for name, t in texts.items():
        p = tmp_path / f"{name}.prototxt"
        p.write_text(t)
        paths.append(p)
    if REF.exists():                                    # the reference's own config files, when present
        for rel in ("examples/mnist/lenet_train_test.prototxt", "examples/cifar10/cifar10_quick_train_test.prototxt",
                    "examples/cifar10/cifar10_full_train_test.prototxt", "models/bvlc_alexnet/train_val.prototxt",
                    "models/bvlc_googlenet/train_val.prototxt",
                    "examples/cifar10/gaussian_failure/solvers/cifar10_vgg11_template.prototxt"):
            if (REF / rel).exists():
                paths.append(REF / rel)
    for p in paths:
        _run(driver, "prototxt", p, n=400)


def test_malformed_files_return_einval_through_the_c_abi(tmp_path):
    """The shipped (unsanitised) librram_caffe.so reports RRAM_EINVAL with a
    message for corrupted weight / state files instead of crashing."""
    from rramsim import caffe
    lib = caffe.load()
    good = (GOLD / "tiny_net.caffemodel").read_bytes()
    cases = {"trunc": good[:len(good) // 2], "ffrun": good[:7] + b"\xff" * 12 + good[7:],
             "biglen": b"\x0a\xff\xff\xff\xff\x0f" + good, "empty_ok": b""}
    for name, data in cases.items():
        p = tmp_path / f"{name}.caffemodel"
        p.write_bytes(data)
        need = ctypes.c_size_t()
        rc = lib.rram_caffemodel_describe(str(p).encode(), None, 0, ctypes.byref(need))
        if name == "empty_ok":
            assert rc == 0                               # an empty NetParameter is valid protobuf
        else:
            assert rc == -1, name                        # RRAM_EINVAL
            assert b"protobuf" in lib.rram_caffe_last_error()
        rc = lib.rram_proto_rewrite(str(p).encode(), str(tmp_path / "out.bin").encode(), 1)
        assert rc in (0, -1)
    bad = tmp_path / "deep.prototxt"
    txt = "layer { " * 500 + "}" * 500
    need = ctypes.c_size_t()
    assert lib.rram_net_describe(txt.encode(), 1, None, 0, ctypes.byref(need)) == -1
    assert b"nesting" in lib.rram_caffe_last_error()
    bad.write_text(txt)
