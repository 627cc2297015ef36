"""The reference's hard-coded pooling vectors (src/caffe/test/test_pooling_layer.cpp).

Each case runs the product's Pooling layer inside a Net (Input -> Pooling,
one top or two with the MAX argmax mask, pooling_layer.hpp:29-33) and checks
the exact expected outputs and masks the reference test writes out:
TestForwardSquare (:49-119), TestForwardRectHigh (:121-244),
TestForwardRectWide (:246-371) with and without the top mask
(TestForwardMax / TestForwardMaxTopMask, :446-457), TestForwardMaxPadded
(:478-521), TestForwardAve (:543-573) and the Setup shape rules (:376-418).
The backward pass routes top diffs to the argmax cells the reference's masks
name (pooling_layer.cu:158-178): with dy = 1 + top index, dx is the scatter-add
of dy over those masks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SQUARE = [[1, 2, 5, 2, 3], [9, 4, 1, 4, 8], [1, 2, 5, 2, 3]]
MAGIC6 = [[35, 1, 6, 26, 19, 24], [3, 32, 7, 21, 23, 25], [31, 9, 2, 22, 27, 20],
          [8, 28, 33, 17, 10, 15], [30, 5, 34, 12, 14, 16], [4, 36, 29, 13, 18, 11]]

CASES = {
    # name: (input plane, pooling_param, (kernel_h, kernel_w), expected output, expected mask)
    "square": (SQUARE, "kernel_size: 2 pool: MAX", (2, 2),
               [[9, 5, 5, 8], [9, 5, 5, 8]],
               [[5, 2, 2, 9], [5, 12, 12, 9]]),
    "rect_high": (MAGIC6, "kernel_h: 3 kernel_w: 2 pool: MAX", (3, 2),
                  [[35, 32, 26, 27, 27], [32, 33, 33, 27, 27], [31, 34, 34, 27, 27], [36, 36, 34, 18, 18]],
                  [[0, 7, 3, 16, 16], [7, 20, 20, 16, 16], [12, 26, 26, 16, 16], [31, 31, 26, 34, 34]]),
    "rect_wide": (MAGIC6, "kernel_h: 2 kernel_w: 3 pool: MAX", (2, 3),
                  [[35, 32, 26, 26], [32, 32, 27, 27], [33, 33, 33, 27], [34, 34, 34, 17], [36, 36, 34, 18]],
                  [[0, 7, 3, 3], [7, 7, 16, 16], [20, 20, 20, 16], [26, 26, 26, 21], [31, 31, 26, 34]]),
}


def _net(shape, pool_param, phase="test", top_mask=False):
    from rramsim import caffe
    dims = " ".join(f"dim: {d}" for d in shape)
    tops = 'top: "y" top: "mask"' if top_mask else 'top: "y"'
    txt = (f'layer {{ name: "x" type: "Input" top: "x" input_param {{ shape {{ {dims} }} }} }}\n'
           f'layer {{ name: "pool" type: "Pooling" bottom: "x" {tops} pooling_param {{ {pool_param} }} }}\n')
    caffe.set_stream_from_torch()
    return caffe.Net(txt, phase)


@pytest.mark.parametrize("top_mask", [False, True])
@pytest.mark.parametrize("case", list(CASES))
def test_forward_max_reference_vectors(device, case, top_mask):
    import torch
    plane, pp, _k, exp_y, exp_m = CASES[case]
    num, channels = 2, 2
    x = np.broadcast_to(np.array(plane, np.float32), (num, channels) + np.array(plane).shape).copy()
    net = _net(x.shape, pp, top_mask=top_mask)
    net.blob("x").copy_(torch.from_numpy(x))
    net.forward()
    y = net.blob("y").cpu().numpy()
    assert y.shape == (num, channels) + np.array(exp_y).shape
    assert np.array_equal(y, np.broadcast_to(np.array(exp_y, np.float32), y.shape))
    if top_mask:
        m = net.blob("mask").cpu().numpy()
        assert np.array_equal(m, np.broadcast_to(np.array(exp_m, np.float32), m.shape))
    net.close()


@pytest.mark.parametrize("case", list(CASES))
def test_backward_max_routes_to_reference_masks(device, case):
    """MAX backward (pooling_layer.cu:158-178) on the reference's inputs:
    every top diff lands on the cell its reference mask names."""
    import torch
    from rramsim import ops
    plane, _pp, (kh, kw), exp_y, exp_m = CASES[case]
    H, W = np.array(plane).shape
    PH, PW = np.array(exp_y).shape
    x = torch.tensor(plane, dtype=torch.float32, device=device).expand(2, 2, H, W).contiguous()
    y = torch.empty(2, 2, PH, PW, device=device)
    mask = torch.empty(2, 2, PH, PW, dtype=torch.int32, device=device)
    geom = (2, 2, H, W, PH, PW, kh, kw, 1, 1, 0, 0)
    ops.pool_fwd(x, y, mask, geom, 0)
    ref_m = np.broadcast_to(np.array(exp_m, np.int32), (2, 2, PH, PW))
    assert np.array_equal(mask.cpu().numpy(), ref_m)
    dy = (1 + torch.arange(2 * 2 * PH * PW, dtype=torch.float32, device=device)).reshape(2, 2, PH, PW)
    dx = torch.full((2, 2, H, W), float("nan"), device=device)
    ops.pool_bwd(dy, mask, dx, geom, 0)
    exp = np.zeros((2, 2, H * W), np.float32)
    dyn = dy.cpu().numpy().reshape(2, 2, -1)
    for n in range(2):
        for c in range(2):
            np.add.at(exp[n, c], ref_m[n, c].reshape(-1), dyn[n, c])
    assert np.array_equal(dx.cpu().numpy().reshape(2, 2, -1), exp)


def test_forward_max_padded(device):                                  # :478-521
    import torch
    x = np.array([[1, 2, 4], [2, 3, 2], [4, 2, 1]], np.float32).reshape(1, 1, 3, 3)
    net = _net(x.shape, "kernel_size: 3 stride: 2 pad: 2 pool: MAX")
    net.blob("x").copy_(torch.from_numpy(x))
    net.forward()
    y = net.blob("y").cpu().numpy()
    assert y.shape == (1, 1, 3, 3)
    np.testing.assert_allclose(y.reshape(3, 3), [[1, 4, 4], [4, 4, 4], [4, 4, 1]], rtol=0, atol=1e-8)
    net.close()


def test_forward_ave(device):                                         # :543-573
    import torch
    net = _net((1, 1, 3, 3), "kernel_size: 3 stride: 1 pad: 1 pool: AVE")
    net.blob("x").copy_(torch.full((1, 1, 3, 3), 2.0))
    net.forward()
    y = net.blob("y").cpu().numpy().reshape(3, 3)
    e, f = 8.0 / 9, 4.0 / 3
    np.testing.assert_allclose(y, [[e, f, e], [f, 2.0, f], [e, f, e]], rtol=0, atol=1e-5)
    net.close()


@pytest.mark.parametrize("pp,exp_hw", [("kernel_size: 3 stride: 2", (3, 2)),                     # TestSetup
                                       ("kernel_size: 3 stride: 2 pad: 1 pool: AVE", (4, 3)),     # TestSetupPadded
                                       ("global_pooling: true pool: AVE", (1, 1))])               # TestSetupGlobalPooling
def test_setup_shapes(device, pp, exp_hw):                            # :376-418
    net = _net((2, 3, 6, 5), pp)
    assert tuple(net.blob("y").shape) == (2, 3) + exp_hw
    net.close()
