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


def test_experiment_solver_like_run_gaussian_exp():
    """run_gaussian_exp.py:50-103 semantics through this build's solver parser
    (caffe.proto defaults applied by rram_solver_describe)."""
    from rramsim import caffe, models, tools
    tpl = models.solver(base_lr=0.005, lr_policy="step", stepsize=10000, gamma=0.1, max_iter=50000,
                        failure_mean=1.0, failure_std=1.0)
    txt = tools.experiment_solver(tpl, 5e6, 1.5e6, threshold=1e-3, remapping="order.txt,50,1000",
                                  genetic="pnet.prototxt,pmodel.caffemodel,300", prob=5, snapshot_prefix="snap")
    rows = caffe.solver_describe(txt)
    fp = [r for r in rows if r[0] == "failure_pattern"]
    assert len(fp) == 1 and fp[0][1:] == ["gaussian", "5000000", "1500000", "5", "90", "5"]
    st = [r[1:] for r in rows if r[0] == "failure_strategy"]
    assert st[0][:2] == ["threshold", "0.001"]
    assert st[1] == ["remapping", "0.001", "1000", "50", "order.txt", "100", "", ""]
    assert st[2] == ["genetic", "0.001", "0", "100", "", "300", "pnet.prototxt", "pmodel.caffemodel"]
    sv = [r for r in rows if r[0] == "solver"][0]
    assert sv[1:] == ["step", "0.005", "50000", "0", "snap/"]
    # defaults with no failure_prob: (10, 20, 10) (caffe.proto:264-268)
    rows = caffe.solver_describe(tools.experiment_solver(tpl, 100.0, 10.0))
    assert [r for r in rows if r[0] == "failure_pattern"][0][4:] == ["10", "20", "10"]
