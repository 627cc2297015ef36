"""HDF5 weight files (src/caffe/util/hdf5.cpp, net.cpp:819-932).

Fixtures are written here with the HDF5 C library itself (libhdf5_hl's
H5LTmake_dataset_* — the calls the reference's hdf5_save_nd_dataset makes),
in the reference's layout: group "data" / layer name / dataset "<blob index>",
optional "diff".  The product reads them through its own loader
(host/hdf5.cpp, C-ABI rram_caffemodel_describe: host-only, no GPU); the GPU
tests round-trip Net::ToHDF5 / CopyTrainedLayersFromHDF5 and the HDF5 solver
snapshots (tests/test_gpu_strategy.py)."""
import ctypes as C
import os

import numpy as np
import pytest

LIBDIRS = [os.environ.get("RRAM_HDF5_LIB_DIR", ""), "/opt/conda/lib", "/usr/lib/x86_64-linux-gnu"]


def _hdf5():
    for d in LIBDIRS:
        for core, hl in (("libhdf5.so", "libhdf5_hl.so"), ("libhdf5.so.103", "libhdf5_hl.so.100")):
            try:
                a = C.CDLL(os.path.join(d, core) if d else core, mode=C.RTLD_GLOBAL)
                b = C.CDLL(os.path.join(d, hl) if d else hl, mode=C.RTLD_GLOBAL)
                return a, b
            except OSError:
                continue
    pytest.skip("libhdf5 not available")


class H5:
    """Minimal ctypes writer/reader over libhdf5 (HDF5 1.10: hid_t = int64)."""

    def __init__(self):
        self.c, self.hl = _hdf5()
        hid, herr = C.c_int64, C.c_int
        self.c.H5open()
        self.c.H5Eset_auto2.argtypes = [hid, C.c_void_p, C.c_void_p]
        self.c.H5Eset_auto2(0, None, None)
        self.c.H5Fcreate.restype = hid
        self.c.H5Fcreate.argtypes = [C.c_char_p, C.c_uint, hid, hid]
        self.c.H5Fopen.restype = hid
        self.c.H5Fopen.argtypes = [C.c_char_p, C.c_uint, hid]
        self.c.H5Fclose.argtypes = [hid]
        self.c.H5Gcreate2.restype = hid
        self.c.H5Gcreate2.argtypes = [hid, C.c_char_p, hid, hid, hid]
        self.c.H5Gclose.argtypes = [hid]
        for fn, ty in (("H5LTmake_dataset_float", C.c_float), ("H5LTmake_dataset_double", C.c_double)):
            f = getattr(self.hl, fn)
            f.restype = herr
            f.argtypes = [hid, C.c_char_p, C.c_int, C.POINTER(C.c_ulonglong), C.POINTER(ty)]
        self.hl.H5LTread_dataset_float.argtypes = [hid, C.c_char_p, C.POINTER(C.c_float)]
        self.hl.H5LTget_dataset_info.argtypes = [hid, C.c_char_p, C.POINTER(C.c_ulonglong), C.POINTER(C.c_int),
                                                 C.POINTER(C.c_size_t)]

    def write_net(self, path, layers, diff=None, double=()):
        f = self.c.H5Fcreate(str(path).encode(), 2, 0, 0)
        assert f >= 0
        for top, content in (("data", layers), ("diff", diff)):
            if content is None:
                continue
            g = self.c.H5Gcreate2(f, top.encode(), 0, 0, 0)
            for name, blobs in content:
                lg = self.c.H5Gcreate2(g, name.encode(), 0, 0, 0)
                for j, arr in enumerate(blobs):
                    dims = (C.c_ulonglong * max(arr.ndim, 1))(*arr.shape)
                    if name in double:
                        a = np.ascontiguousarray(arr, np.float64)
                        rc = self.hl.H5LTmake_dataset_double(lg, str(j).encode(), arr.ndim, dims,
                                                             a.ctypes.data_as(C.POINTER(C.c_double)))
                    else:
                        a = np.ascontiguousarray(arr, np.float32)
                        rc = self.hl.H5LTmake_dataset_float(lg, str(j).encode(), arr.ndim, dims,
                                                            a.ctypes.data_as(C.POINTER(C.c_float)))
                    assert rc >= 0
                self.c.H5Gclose(lg)
            self.c.H5Gclose(g)
        self.c.H5Fclose(f)

    def read(self, path, name):
        f = self.c.H5Fopen(str(path).encode(), 0, 0)
        assert f >= 0
        dims = (C.c_ulonglong * 8)()
        cls, sz = C.c_int(), C.c_size_t()
        assert self.hl.H5LTget_dataset_info(f, name.encode(), dims, C.byref(cls), C.byref(sz)) >= 0
        ndims = C.c_int()
        self.hl.H5LTget_dataset_ndims.argtypes = [C.c_int64, C.c_char_p, C.POINTER(C.c_int)]
        self.hl.H5LTget_dataset_ndims(f, name.encode(), C.byref(ndims))
        shape = tuple(dims[i] for i in range(ndims.value))
        out = np.empty(int(np.prod(shape)) if shape else 1, np.float32)
        assert self.hl.H5LTread_dataset_float(f, name.encode(), out.ctypes.data_as(C.POINTER(C.c_float))) >= 0
        self.c.H5Fclose(f)
        return out.reshape(shape)


def test_reference_layout_read_by_the_product(tmp_path):
    from rramsim import caffe
    h = H5()
    rng = np.random.default_rng(3)
    conv_w = rng.standard_normal((20, 1, 5, 5)).astype(np.float32)
    conv_b = rng.standard_normal(20).astype(np.float32)
    ip_w = rng.standard_normal((10, 50)).astype(np.float32)
    ip_b = rng.standard_normal(10)                    # stored as double: read back as float (hdf5.cpp:67-83)
    p = tmp_path / "ref.caffemodel.h5"
    h.write_net(p, [("conv1", [conv_w, conv_b]), ("pool1", []), ("ip2", [ip_w, ip_b])],
                diff=[("conv1", [conv_w * 0, conv_b * 0 + 1])], double=("ip2",))
    rows = {(r[0], r[2]): r for r in caffe.caffemodel_describe(str(p))}
    assert rows[("conv1", 0)][3] == (20, 1, 5, 5) and rows[("conv1", 0)][4] == 500
    assert abs(rows[("conv1", 0)][5] - float(conv_w.astype(np.float64).sum())) < 1e-3
    assert rows[("conv1", 1)][6] == 20                 # diff present for conv1
    assert rows[("ip2", 1)][3] == (10,) and abs(rows[("ip2", 1)][5] - float(ip_b.astype(np.float32).sum())) < 1e-4
    assert rows[("pool1", -1)][4] == 0                 # a layer group without blobs


def test_corrupt_or_missing_h5_is_einval(tmp_path):
    from rramsim import RramError, caffe
    H5()                                              # skip when libhdf5 is absent
    bad = tmp_path / "bad.caffemodel.h5"
    bad.write_bytes(b"\x89HDF\r\n\x1a\n" + b"\x00" * 40)
    with pytest.raises(RramError):
        caffe.caffemodel_describe(str(bad))
    with pytest.raises(RramError, match="Couldn't open"):
        caffe.caffemodel_describe(str(tmp_path / "missing.caffemodel.h5"))
    h = H5()                                          # a valid HDF5 file without the "data" group
    f = h.c.H5Fcreate(str(tmp_path / "empty.caffemodel.h5").encode(), 2, 0, 0)
    h.c.H5Fclose(f)
    with pytest.raises(RramError, match="Error reading weights"):
        caffe.caffemodel_describe(str(tmp_path / "empty.caffemodel.h5"))


@pytest.mark.gpu
def test_net_hdf5_round_trip_and_reference_layout(device, tmp_path):
    """Net::ToHDF5 writes the reference's layout (read back here with libhdf5
    directly) and CopyTrainedLayersFromHDF5 restores every param bit for bit."""
    import torch
    from rramsim import caffe, models
    h = H5()
    caffe.set_stream_from_torch()
    caffe.set_random_seed(11)
    a = caffe.Net(models.lenet(train_batch=8), "train", models.net_options("lenet"))
    path = tmp_path / "lenet.caffemodel.h5"
    for p in a.params():
        p["diff"].copy_(torch.randn_like(p["diff"]))
    a.save(str(path), write_diff=True)
    ps = a.params()
    np.testing.assert_array_equal(h.read(path, "data/conv1/0").reshape(-1), ps[0]["data"].cpu().numpy())
    assert h.read(path, "data/conv1/0").shape == (20, 1, 5, 5)
    np.testing.assert_array_equal(h.read(path, "diff/ip1/1"), ps[5]["diff"].cpu().numpy())
    caffe.set_random_seed(12)
    b = caffe.Net(models.lenet(train_batch=8), "train", models.net_options("lenet"))
    assert not torch.equal(b.params()[0]["data"], ps[0]["data"])
    b.copy_from(str(path))
    for x, y in zip(ps, b.params()):
        assert torch.equal(x["data"], y["data"])
    a.close()
    b.close()
