"""The last reference-held known answers of the GEMM / InnerProduct /
Convolution path, run through the product's C-ABI and Layer API.

* GEMV KAT (src/caffe/test/test_util_blas.cpp:91-125): A = [1 2 3; 4 5 6],
  A·[1 2 3] = {14, 32} and Aᵀ·[1 2] = {9, 12, 15}, exact (EXPECT_EQ); and the
  same {14, 32} through rram_ip_fwd at M = 1, the shape the reference routes
  through caffe_gpu_gemv (inner_product_layer.cu:15-20).
* InnerProduct (src/caffe/test/test_inner_product_layer.cpp; bottom 2x3x4x5
  and 1x2x3x4 uniform [0,1], num_output 10, uniform weights, bias in [1,2]):
  TestForward (:107-136, every output >= 1), TestForwardTranspose (:145-210:
  a transpose: true layer with the transposed weights gives the same top,
  EXPECT_FLOAT_EQ), TestForwardNoBatch (:211-240), TestBackwardTranspose
  (:295-386: weight diffs equal transposed, bottom diffs equal, all non-zero).
* TestSobelConvolution (src/caffe/test/test_convolution_layer.cpp:498-590):
  the 3x3 stride-2 Sobel G_x filter over 3 channels equals the separable
  [1 2 1]ᵀ (3x1, stride 2x1) then [-1 0 1] (1x3, stride 1x2) pair within
  1e-4, on the test's 2x3x6x4 Gaussian bottom (:156-166), no bias.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def ulps_equal(a, b, ulps=4):
    """gtest EXPECT_FLOAT_EQ: within 4 units in the last place."""
    a = np.asarray(a, np.float32).ravel()
    b = np.asarray(b, np.float32).ravel()
    ia = a.view(np.int32).astype(np.int64)
    ib = b.view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, -(ia & 0x7FFFFFFF), ia)        # sign-magnitude -> biased order
    ib = np.where(ib < 0, -(ib & 0x7FFFFFFF), ib)
    return bool(np.all(np.abs(ia - ib) <= ulps))


# ------------------------------------------------------------------ GEMV KAT
def test_gemv_kat(device):
    import torch
    from rramsim import ops
    A = torch.tensor([1, 2, 3, 4, 5, 6], dtype=torch.float32, device=device)
    x = torch.tensor([1, 2, 3], dtype=torch.float32, device=device)
    y = torch.full((2,), float("nan"), device=device)
    ops.gemv(False, 2, 3, 1.0, A, x, 0.0, y)                   # beta 0: the NaN in y is not read
    assert y.cpu().tolist() == [14.0, 32.0]
    y2 = torch.tensor([1, 2], dtype=torch.float32, device=device)
    x2 = torch.full((3,), float("nan"), device=device)
    ops.gemv(True, 2, 3, 1.0, A, y2, 0.0, x2)
    assert x2.cpu().tolist() == [9.0, 12.0, 15.0]
    # alpha / beta (caffe_gpu_gemv's full form): y = 2 A x + 3 y
    y3 = torch.tensor([1, -1], dtype=torch.float32, device=device)
    ops.gemv(False, 2, 3, 2.0, A, x, 3.0, y3)
    assert y3.cpu().tolist() == [31.0, 61.0]


def test_ip_forward_m1_is_the_gemv_kat(device):
    """rram_ip_fwd at M = 1 (the reference's gemv route): W = [1 2 3; 4 5 6]
    (N = 2, K = 3), x = [1 2 3], bias [0.5, -1] -> {14.5, 31}, exact; with
    the fused ReLU and a negative bias the clamp applies."""
    import torch
    from rramsim import ops
    W = torch.tensor([[1, 2, 3], [4, 5, 6]], dtype=torch.float32, device=device)
    x = torch.tensor([[1, 2, 3]], dtype=torch.float32, device=device)
    b = torch.tensor([0.5, -1.0], device=device)
    y = torch.full((1, 2), float("nan"), device=device)
    ops.ip_fwd(x, W, b, y, 1, 2, 3)
    assert y.cpu().tolist() == [[14.5, 31.0]]
    ops.ip_fwd(x, W, torch.tensor([0.0, -40.0], device=device), y, 1, 2, 3, relu=True)
    assert y.cpu().tolist() == [[14.0, 0.0]]
    ops.ip_fwd(x, W, None, y, 1, 2, 3)
    assert y.cpu().tolist() == [[14.0, 32.0]]


# -------------------------------------------------------------- InnerProduct
def _ip_net(shape, transpose, num_output=10):
    from rramsim import caffe
    dims = " ".join(f"dim: {d}" for d in shape)
    txt = (f'force_backward: true\n'
           f'layer {{ name: "x" type: "Input" top: "x" input_param {{ shape {{ {dims} }} }} }}\n'
           f'layer {{ name: "ip" type: "InnerProduct" bottom: "x" top: "y" inner_product_param {{ '
           f'num_output: {num_output} transpose: {"true" if transpose else "false"} '
           f'weight_filler {{ type: "uniform" }} bias_filler {{ type: "uniform" min: 1 max: 2 }} }} }}\n')
    caffe.set_stream_from_torch()
    return caffe.Net(txt, "train")


def _bottom(shape, seed=1701):
    return np.random.default_rng(seed).uniform(0, 1, shape).astype(np.float32)   # UniformFiller [0, 1]


@pytest.mark.parametrize("shape", [(2, 3, 4, 5), (1, 2, 3, 4)], ids=["TestForward", "TestForwardNoBatch"])
def test_ip_forward_outputs_at_least_one(device, shape):
    import torch
    from _ref64 import check_ip
    net = _ip_net(shape, False)
    x = _bottom(shape)
    net.blob("x").copy_(torch.from_numpy(x))
    net.forward()
    y = net.blob("y").cpu().numpy()
    assert y.shape == (shape[0], 10)
    assert (y >= 1.0).all()
    ps = net.params()
    w = ps[0]["data"].cpu().numpy().reshape(10, -1)
    b = ps[1]["data"].cpu().numpy()
    assert (w >= 0).all() and (w <= 1).all() and (b >= 1).all() and (b <= 2).all()
    check_ip(y, x.reshape(shape[0], -1), w, b, what=f"ip {shape}")
    net.close()


def test_ip_forward_transpose(device):
    import torch
    shape = (2, 3, 4, 5)
    x = torch.from_numpy(_bottom(shape))
    net = _ip_net(shape, False)
    net.blob("x").copy_(x)
    net.forward()
    top = net.blob("y").cpu().numpy()
    ps = net.params()
    w = ps[0]["data"].cpu().numpy().reshape(10, 60)
    b = ps[1]["data"].cpu().numpy()
    net_t = _ip_net(shape, True)
    pt = net_t.params()
    assert pt[0]["data"].numel() == w.size                    # blobs()[0] is [K][N] = [60][10]
    pt[0]["data"].copy_(torch.from_numpy(np.ascontiguousarray(w.T)).reshape(-1))
    pt[1]["data"].copy_(torch.from_numpy(b))
    net_t.blob("x").copy_(x)
    net_t.forward()
    top_t = net_t.blob("y").cpu().numpy()
    assert top_t.shape == top.shape
    assert ulps_equal(top, top_t), np.abs(top - top_t).max()
    net.close()
    net_t.close()


def test_ip_backward_transpose(device):
    import torch
    shape = (2, 3, 4, 5)
    x = torch.from_numpy(_bottom(shape))
    diff = torch.from_numpy(np.random.default_rng(7).uniform(0, 1, (2, 10)).astype(np.float32))
    net = _ip_net(shape, False)
    net.blob("x").copy_(x)
    net.forward()
    net.blob("y", diff=True).copy_(diff)
    net.backward()
    ps = net.params()
    w = ps[0]["data"].cpu().numpy().reshape(10, 60)
    dw = ps[0]["diff"].cpu().numpy().reshape(10, 60)
    dx = net.blob("x", diff=True).cpu().numpy()
    net_t = _ip_net(shape, True)
    pt = net_t.params()
    pt[0]["data"].copy_(torch.from_numpy(np.ascontiguousarray(w.T)).reshape(-1))
    pt[1]["data"].copy_(ps[1]["data"])
    net_t.blob("x").copy_(x)
    net_t.forward()
    net_t.blob("y", diff=True).copy_(diff)
    net_t.backward()
    dw_t = pt[0]["diff"].cpu().numpy().reshape(60, 10)
    dx_t = net_t.blob("x", diff=True).cpu().numpy()
    assert (dw != 0).all() and (dx != 0).all()
    assert ulps_equal(dw, dw_t.T), np.abs(dw - dw_t.T).max()
    assert ulps_equal(dx, dx_t), np.abs(dx - dx_t).max()
    # and against float64 (dW = dYᵀ X, dX = dY W)
    xd = x.numpy().reshape(2, 60).astype(np.float64)
    np.testing.assert_allclose(dw, diff.numpy().T.astype(np.float64) @ xd, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(dx.reshape(2, 60), diff.numpy().astype(np.float64) @ w, rtol=1e-5, atol=1e-6)
    net.close()
    net_t.close()


# ------------------------------------------------------------------- Sobel
def _conv_net(shape, conv_param):
    from rramsim import caffe
    dims = " ".join(f"dim: {d}" for d in shape)
    txt = (f'layer {{ name: "x" type: "Input" top: "x" input_param {{ shape {{ {dims} }} }} }}\n'
           f'layer {{ name: "conv" type: "Convolution" bottom: "x" top: "y" convolution_param {{ '
           f'num_output: 1 bias_term: false {conv_param} }} }}\n')
    caffe.set_stream_from_torch()
    return caffe.Net(txt, "test")


def _run_conv(shape, conv_param, weights, x):
    import torch
    net = _conv_net(shape, conv_param)
    p = net.params()
    assert len(p) == 1                                         # bias_term: false
    p[0]["data"].copy_(torch.tensor(np.asarray(weights, np.float32).ravel()))
    net.blob("x").copy_(torch.from_numpy(x))
    net.forward()
    y = net.blob("y").cpu().numpy()
    net.close()
    return y


def test_sobel_convolution(device):
    x = np.random.default_rng(1701).standard_normal((2, 3, 6, 4)).astype(np.float32)   # GaussianFiller
    sobel = np.tile(np.array([-1, 0, 1, -2, 0, 2, -1, 0, 1], np.float32), 3)           # :517-529
    y = _run_conv((2, 3, 6, 4), "kernel_size: 3 stride: 2", sobel, x)
    assert y.shape == (2, 1, 2, 1)
    col = _run_conv((2, 3, 6, 4), "kernel_h: 3 kernel_w: 1 stride_h: 2 stride_w: 1",
                    np.tile(np.array([1, 2, 1], np.float32), 3), x)                    # :545-553
    assert col.shape == (2, 1, 2, 4)
    sep = _run_conv(col.shape, "kernel_h: 1 kernel_w: 3 stride_h: 1 stride_w: 2", [-1, 0, 1], col)   # :567-573
    assert sep.shape == y.shape
    np.testing.assert_allclose(y, sep, rtol=0, atol=1e-4)                               # EXPECT_NEAR 1e-4
    # both against the direct float64 G_x
    ref = np.zeros((2, 1, 2, 1))
    k = sobel.reshape(3, 3, 3).astype(np.float64)
    for n in range(2):
        for i in range(2):
            ref[n, 0, i, 0] = (x[n, :, 2 * i:2 * i + 3, 0:3].astype(np.float64) * k).sum()
    np.testing.assert_allclose(y, ref, rtol=0, atol=1e-4)
