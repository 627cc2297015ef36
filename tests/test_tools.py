"""CPU tests of the experiment tools (prune_order.py restated, §8f-4)."""
import numpy as np


def test_prune_orders_hand_example(tmp_path):
    from rramsim import tools
    w1 = np.array([[0.5, -0.1, 0.3],
                   [0.05, 0.9, -0.02],
                   [0.7, 0.6, 0.8],
                   [-0.01, 0.03, 0.2]], np.float32)      # 4 neurons x 3 inputs
    w2 = np.array([[0.4, 0.02, 0.9, 0.01],
                   [-0.3, 0.5, 0.04, 0.6]], np.float32)   # 2 outputs x 4 neurons
    pruned, orders = tools.prune_orders([w1, w2], 0.5)
    # half of each layer's weights (smallest |w|) are zeroed
    assert (pruned[0] == 0).sum() == 6 and (pruned[1] == 0).sum() == 4
    # |w1| sorted: 0.01(9) 0.02(5) 0.03(10) 0.05(3) 0.1(1) 0.2(11) are the six smallest
    assert set(np.flatnonzero(pruned[0].ravel() == 0)) == {9, 5, 10, 3, 1, 11}
    zeros = (pruned[0] == 0).sum(1) + (pruned[1] == 0).sum(0)
    assert list(orders[0]) == list(np.argsort(zeros))
    # neuron 2 keeps all its inputs and output weights -> sorted first
    assert orders[0][0] == 2
    f = tmp_path / "order.txt"
    tools.write_prune_order_file(str(f), orders)
    assert f.read_text().split() == [str(x) for x in orders[0]]


def test_magnitude_prune_ratio_edges():
    from rramsim import tools
    w = np.arange(1, 11, dtype=np.float32).reshape(2, 5)
    assert np.array_equal(tools.magnitude_prune(w, 0.0), w)
    assert not tools.magnitude_prune(w, 1.0).any()
    p = tools.magnitude_prune(-w, 0.3)              # int(10 * 0.3) = 3 smallest |w|
    assert np.array_equal(p.ravel()[:3], [0, 0, 0]) and (p.ravel()[3:] != 0).all()
