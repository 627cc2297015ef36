"""Network definitions of the benchmark configs, emitted as Caffe prototxt.

The reference keeps these nets as .prototxt files under examples/ and models/
(lenet_train_test, cifar10_quick_train_test, cifar10_full_train_test,
bvlc_alexnet/train_val, bvlc_reference_caffenet/train_val,
bvlc_googlenet/train_val).  They are regenerated here layer for layer (same
layer names, types, geometry, fillers and lr/decay multipliers) so the
C++ parser consumes them exactly as it would the reference files; the data
layers stay `Data` and become synthetic tensors of the configured shape
(LMDB sources are out of scope).  tests/test_models.py checks each generated
net against the reference prototxt's parsed layer table when the reference
tree is available.
"""
from __future__ import annotations

from typing import List, Optional


class _P:
    """Tiny prototxt builder."""

    def __init__(self, name: str):
        self.lines: List[str] = [f'name: "{name}"']

    @staticmethod
    def _fmt(v):
        if isinstance(v, bool):
            return "true" if v else "false"
        if isinstance(v, str):
            return v if v.isupper() or v in ("true", "false") else f'"{v}"'
        return repr(v) if isinstance(v, float) else str(v)

    @classmethod
    def _block(cls, key, d, ind):
        pad = "  " * ind
        out = [f"{pad}{key} {{"]
        for k, v in d.items():
            items = v if isinstance(v, list) else [v]
            for it in items:
                if isinstance(it, dict):
                    out += cls._block(k, it, ind + 1)
                else:
                    out.append(f"{pad}  {k}: {cls._fmt(it)}")
        out.append(f"{pad}}}")
        return out

    def layer(self, **d):
        self.lines += self._block("layer", d, 0)

    def text(self):
        return "\n".join(self.lines) + "\n"


W1B2 = [dict(lr_mult=1, decay_mult=1), dict(lr_mult=2, decay_mult=0)]
W1B2_NODECAY = [dict(lr_mult=1), dict(lr_mult=2)]


def _data(p, scale=None, mean=False, crop=None, train_batch=64, test_batch=100, phases=("TRAIN", "TEST"),
          name="data"):
    for ph, bs in zip(("TRAIN", "TEST"), (train_batch, test_batch)):
        if ph not in phases:
            continue
        tp = {}
        if scale is not None:
            tp["scale"] = scale
        if crop is not None:
            tp["mirror"] = ph == "TRAIN"
            tp["crop_size"] = crop
        if mean:
            tp["mean_file"] = "mean.binaryproto"
        d = dict(name=name, type="Data",
                 top=["data", "label"], include=dict(phase=ph))
        if tp:
            d["transform_param"] = tp
        d["data_param"] = dict(source=f"synthetic_{ph.lower()}", batch_size=bs, backend="LMDB")
        p.layer(**d)


def _conv(p, name, bottom, n, k, s=1, pad=0, group=1, wf=None, bf=None, param=None, top=None):
    cp = dict(num_output=n)
    if pad:
        cp["pad"] = pad
    cp["kernel_size"] = k
    if s != 1:
        cp["stride"] = s
    if group != 1:
        cp["group"] = group
    cp["weight_filler"] = wf or dict(type="xavier")
    cp["bias_filler"] = bf or dict(type="constant")
    d = dict(name=name, type="Convolution", bottom=bottom, top=top or name)
    if param:
        d["param"] = param
    d["convolution_param"] = cp
    p.layer(**d)


def _ip(p, name, bottom, n, wf=None, bf=None, param=None):
    d = dict(name=name, type="InnerProduct", bottom=bottom, top=name)
    if param:
        d["param"] = param
    d["inner_product_param"] = dict(num_output=n, weight_filler=wf or dict(type="xavier"),
                                    bias_filler=bf or dict(type="constant"))
    p.layer(**d)


def _pool(p, name, bottom, pool, k, s, pad=0, top=None):
    pp = dict(pool=pool, kernel_size=k, stride=s)
    if pad:
        pp["pad"] = pad
    p.layer(name=name, type="Pooling", bottom=bottom, top=top or name, pooling_param=pp)


def _relu(p, name, blob):
    p.layer(name=name, type="ReLU", bottom=blob, top=blob)


def _lrn(p, name, bottom, size, alpha, beta, region=None):
    lp = dict(local_size=size, alpha=alpha, beta=beta)
    if region:
        lp["norm_region"] = region
    p.layer(name=name, type="LRN", bottom=bottom, top=name, lrn_param=lp)


def _heads(p, bottom, acc_top5=False):
    p.layer(name="accuracy", type="Accuracy", bottom=[bottom, "label"], top="accuracy",
            include=dict(phase="TEST"))
    if acc_top5:
        p.layer(name="accuracy_top5", type="Accuracy", bottom=[bottom, "label"], top="accuracy_top5",
                include=dict(phase="TEST"), accuracy_param=dict(top_k=5))
    p.layer(name="loss", type="SoftmaxWithLoss", bottom=[bottom, "label"], top="loss")


# ----------------------------------------------------------------- configs
def lenet(train_batch=64, test_batch=100) -> str:
    """examples/mnist/lenet_train_test.prototxt (C1)."""
    p = _P("LeNet")
    _data(p, scale=0.00390625, train_batch=train_batch, test_batch=test_batch, name="mnist")
    _conv(p, "conv1", "data", 20, 5, param=W1B2_NODECAY)
    _pool(p, "pool1", "conv1", "MAX", 2, 2)
    _conv(p, "conv2", "pool1", 50, 5, param=W1B2_NODECAY)
    _pool(p, "pool2", "conv2", "MAX", 2, 2)
    _ip(p, "ip1", "pool2", 500, param=W1B2_NODECAY)
    _relu(p, "relu1", "ip1")
    _ip(p, "ip2", "ip1", 10, param=W1B2_NODECAY)
    _heads(p, "ip2")
    return p.text()


def cifar10_quick(train_batch=100, test_batch=100) -> str:
    """examples/cifar10/cifar10_quick_train_test.prototxt (C2)."""
    p = _P("CIFAR10_quick")
    _data(p, mean=True, train_batch=train_batch, test_batch=test_batch, name="cifar")
    g = lambda s: dict(type="gaussian", std=s)  # noqa: E731
    _conv(p, "conv1", "data", 32, 5, pad=2, wf=g(0.0001), param=W1B2_NODECAY)
    _pool(p, "pool1", "conv1", "MAX", 3, 2)
    _relu(p, "relu1", "pool1")
    _conv(p, "conv2", "pool1", 32, 5, pad=2, wf=g(0.01), param=W1B2_NODECAY)
    _relu(p, "relu2", "conv2")
    _pool(p, "pool2", "conv2", "AVE", 3, 2)
    _conv(p, "conv3", "pool2", 64, 5, pad=2, wf=g(0.01), param=W1B2_NODECAY)
    _relu(p, "relu3", "conv3")
    _pool(p, "pool3", "conv3", "AVE", 3, 2)
    _ip(p, "ip1", "pool3", 64, wf=g(0.1), param=W1B2_NODECAY)
    _ip(p, "ip2", "ip1", 10, wf=g(0.1), param=W1B2_NODECAY)
    _heads(p, "ip2")
    return p.text()


def cifar10_full(train_batch=100, test_batch=100) -> str:
    """examples/cifar10/cifar10_full_train_test.prototxt (C4)."""
    p = _P("CIFAR10_full")
    _data(p, mean=True, train_batch=train_batch, test_batch=test_batch, name="cifar")
    g = lambda s: dict(type="gaussian", std=s)  # noqa: E731
    _conv(p, "conv1", "data", 32, 5, pad=2, wf=g(0.0001), param=W1B2_NODECAY)
    _pool(p, "pool1", "conv1", "MAX", 3, 2)
    _relu(p, "relu1", "pool1")
    _lrn(p, "norm1", "pool1", 3, 5e-05, 0.75, "WITHIN_CHANNEL")
    _conv(p, "conv2", "norm1", 32, 5, pad=2, wf=g(0.01), param=W1B2_NODECAY)
    _relu(p, "relu2", "conv2")
    _pool(p, "pool2", "conv2", "AVE", 3, 2)
    _lrn(p, "norm2", "pool2", 3, 5e-05, 0.75, "WITHIN_CHANNEL")
    _conv(p, "conv3", "norm2", 64, 5, pad=2, wf=g(0.01))
    _relu(p, "relu3", "conv3")
    _pool(p, "pool3", "conv3", "AVE", 3, 2)
    _ip(p, "ip1", "pool3", 10, wf=g(0.01), param=[dict(lr_mult=1, decay_mult=250), dict(lr_mult=2, decay_mult=0)])
    _heads(p, "ip1")
    return p.text()


def alexnet(train_batch=256, test_batch=256, caffenet=False) -> str:
    """models/bvlc_alexnet/train_val.prototxt (C3); caffenet=True gives
    models/bvlc_reference_caffenet/train_val.prototxt (pool before norm).
    The reference's TEST batch is 50; the benchmark config uses 256."""
    p = _P("CaffeNet" if caffenet else "AlexNet")
    _data(p, mean=True, crop=227, train_batch=train_batch, test_batch=test_batch)
    g = lambda s: dict(type="gaussian", std=s)  # noqa: E731
    c = lambda v: dict(type="constant", value=v)  # noqa: E731
    _conv(p, "conv1", "data", 96, 11, s=4, wf=g(0.01), bf=c(0), param=W1B2)
    _relu(p, "relu1", "conv1")
    if caffenet:
        _pool(p, "pool1", "conv1", "MAX", 3, 2)
        _lrn(p, "norm1", "pool1", 5, 0.0001, 0.75)
        nxt = "norm1"
    else:
        _lrn(p, "norm1", "conv1", 5, 0.0001, 0.75)
        _pool(p, "pool1", "norm1", "MAX", 3, 2)
        nxt = "pool1"
    _conv(p, "conv2", nxt, 256, 5, pad=2, group=2, wf=g(0.01), bf=c(0.1 if not caffenet else 1), param=W1B2)
    _relu(p, "relu2", "conv2")
    if caffenet:
        _pool(p, "pool2", "conv2", "MAX", 3, 2)
        _lrn(p, "norm2", "pool2", 5, 0.0001, 0.75)
        nxt = "norm2"
    else:
        _lrn(p, "norm2", "conv2", 5, 0.0001, 0.75)
        _pool(p, "pool2", "norm2", "MAX", 3, 2)
        nxt = "pool2"
    _conv(p, "conv3", nxt, 384, 3, pad=1, wf=g(0.01), bf=c(0), param=W1B2)
    _relu(p, "relu3", "conv3")
    _conv(p, "conv4", "conv3", 384, 3, pad=1, group=2, wf=g(0.01), bf=c(0.1 if not caffenet else 1), param=W1B2)
    _relu(p, "relu4", "conv4")
    _conv(p, "conv5", "conv4", 256, 3, pad=1, group=2, wf=g(0.01), bf=c(0.1 if not caffenet else 1), param=W1B2)
    _relu(p, "relu5", "conv5")
    _pool(p, "pool5", "conv5", "MAX", 3, 2)
    _ip(p, "fc6", "pool5", 4096, wf=g(0.005), bf=c(0.1 if not caffenet else 1), param=W1B2)
    _relu(p, "relu6", "fc6")
    p.layer(name="drop6", type="Dropout", bottom="fc6", top="fc6", dropout_param=dict(dropout_ratio=0.5))
    _ip(p, "fc7", "fc6", 4096, wf=g(0.005), bf=c(0.1 if not caffenet else 1), param=W1B2)
    _relu(p, "relu7", "fc7")
    p.layer(name="drop7", type="Dropout", bottom="fc7", top="fc7", dropout_param=dict(dropout_ratio=0.5))
    _ip(p, "fc8", "fc7", 1000, wf=g(0.01), bf=c(0), param=W1B2)
    _heads(p, "fc8")
    return p.text()


def _inception(p, name, bottom, c1, c3r, c3, c5r, c5, pp):
    x = dict(type="xavier")
    c = dict(type="constant", value=0.2)
    b = f"inception_{name}"
    _conv(p, f"{b}/1x1", bottom, c1, 1, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_1x1", f"{b}/1x1")
    _conv(p, f"{b}/3x3_reduce", bottom, c3r, 1, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_3x3_reduce", f"{b}/3x3_reduce")
    _conv(p, f"{b}/3x3", f"{b}/3x3_reduce", c3, 3, pad=1, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_3x3", f"{b}/3x3")
    _conv(p, f"{b}/5x5_reduce", bottom, c5r, 1, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_5x5_reduce", f"{b}/5x5_reduce")
    _conv(p, f"{b}/5x5", f"{b}/5x5_reduce", c5, 5, pad=2, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_5x5", f"{b}/5x5")
    _pool(p, f"{b}/pool", bottom, "MAX", 3, 1, pad=1)
    _conv(p, f"{b}/pool_proj", f"{b}/pool", pp, 1, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_pool_proj", f"{b}/pool_proj")
    p.layer(name=f"{b}/output", type="Concat",
            bottom=[f"{b}/1x1", f"{b}/3x3", f"{b}/5x5", f"{b}/pool_proj"], top=f"{b}/output")
    return f"{b}/output"


def _aux(p, idx, bottom):
    x = dict(type="xavier")
    c = dict(type="constant", value=0.2)
    b = f"loss{idx}"
    _pool(p, f"{b}/ave_pool", bottom, "AVE", 5, 3)
    _conv(p, f"{b}/conv", f"{b}/ave_pool", 128, 1, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_conv", f"{b}/conv")
    _ip(p, f"{b}/fc", f"{b}/conv", 1024, wf=x, bf=c, param=W1B2)
    _relu(p, f"{b}/relu_fc", f"{b}/fc")
    p.layer(name=f"{b}/drop_fc", type="Dropout", bottom=f"{b}/fc", top=f"{b}/fc",
            dropout_param=dict(dropout_ratio=0.7))
    _ip(p, f"{b}/classifier", f"{b}/fc", 1000, wf=x, bf=dict(type="constant", value=0), param=W1B2)
    # the reference names both auxiliary loss tops "loss<k>/loss1"
    # (models/bvlc_googlenet/train_val.prototxt), kept for log parity
    p.layer(name=f"{b}/loss", type="SoftmaxWithLoss", bottom=[f"{b}/classifier", "label"],
            top=f"{b}/loss1", loss_weight=0.3)
    p.layer(name=f"{b}/top-1", type="Accuracy", bottom=[f"{b}/classifier", "label"], top=f"{b}/top-1",
            include=dict(phase="TEST"))
    p.layer(name=f"{b}/top-5", type="Accuracy", bottom=[f"{b}/classifier", "label"], top=f"{b}/top-5",
            include=dict(phase="TEST"), accuracy_param=dict(top_k=5))


def googlenet(train_batch=32, test_batch=256) -> str:
    """models/bvlc_googlenet/train_val.prototxt (C5; reference TEST batch 50,
    benchmark batch 256), including the two auxiliary classifiers."""
    p = _P("GoogleNet")
    _data(p, mean=True, crop=224, train_batch=train_batch, test_batch=test_batch)
    x = dict(type="xavier")
    c = dict(type="constant", value=0.2)
    _conv(p, "conv1/7x7_s2", "data", 64, 7, s=2, pad=3, wf=x, bf=c, param=W1B2)
    _relu(p, "conv1/relu_7x7", "conv1/7x7_s2")
    _pool(p, "pool1/3x3_s2", "conv1/7x7_s2", "MAX", 3, 2)
    _lrn(p, "pool1/norm1", "pool1/3x3_s2", 5, 0.0001, 0.75)
    _conv(p, "conv2/3x3_reduce", "pool1/norm1", 64, 1, wf=x, bf=c, param=W1B2)
    _relu(p, "conv2/relu_3x3_reduce", "conv2/3x3_reduce")
    _conv(p, "conv2/3x3", "conv2/3x3_reduce", 192, 3, pad=1, wf=x, bf=c, param=W1B2)
    _relu(p, "conv2/relu_3x3", "conv2/3x3")
    _lrn(p, "conv2/norm2", "conv2/3x3", 5, 0.0001, 0.75)
    _pool(p, "pool2/3x3_s2", "conv2/norm2", "MAX", 3, 2)
    t = _inception(p, "3a", "pool2/3x3_s2", 64, 96, 128, 16, 32, 32)
    t = _inception(p, "3b", t, 128, 128, 192, 32, 96, 64)
    _pool(p, "pool3/3x3_s2", t, "MAX", 3, 2)
    t = _inception(p, "4a", "pool3/3x3_s2", 192, 96, 208, 16, 48, 64)
    _aux(p, 1, t)
    t = _inception(p, "4b", t, 160, 112, 224, 24, 64, 64)
    t = _inception(p, "4c", t, 128, 128, 256, 24, 64, 64)
    t = _inception(p, "4d", t, 112, 144, 288, 32, 64, 64)
    _aux(p, 2, t)
    t = _inception(p, "4e", t, 256, 160, 320, 32, 128, 128)
    _pool(p, "pool4/3x3_s2", t, "MAX", 3, 2)
    t = _inception(p, "5a", "pool4/3x3_s2", 256, 160, 320, 32, 128, 128)
    t = _inception(p, "5b", t, 384, 192, 384, 48, 128, 128)
    _pool(p, "pool5/7x7_s1", t, "AVE", 7, 1)
    p.layer(name="pool5/drop_7x7_s1", type="Dropout", bottom="pool5/7x7_s1", top="pool5/7x7_s1",
            dropout_param=dict(dropout_ratio=0.4))
    _ip(p, "loss3/classifier", "pool5/7x7_s1", 1000, wf=x, bf=dict(type="constant", value=0), param=W1B2)
    p.layer(name="loss3/loss3", type="SoftmaxWithLoss", bottom=["loss3/classifier", "label"], top="loss3/loss3",
            loss_weight=1)
    p.layer(name="loss3/top-1", type="Accuracy", bottom=["loss3/classifier", "label"], top="loss3/top-1",
            include=dict(phase="TEST"))
    p.layer(name="loss3/top-5", type="Accuracy", bottom=["loss3/classifier", "label"], top="loss3/top-5",
            include=dict(phase="TEST"), accuracy_param=dict(top_k=5))
    return p.text()


def solver(base_lr=0.01, momentum=0.9, weight_decay=0.0005, lr_policy="fixed", max_iter=100, test_iter=1,
           test_interval=0, display=0, gamma=None, power=None, stepsize=None, random_seed=1701,
           failure_mean: Optional[float] = None, failure_std: Optional[float] = None, failure_prob=None,
           threshold: Optional[float] = None, test_initialization=False, average_loss: Optional[int] = None) -> str:
    """SolverParameter text with the fork's failure_pattern / failure_strategy
    blocks (caffe.proto:244-290), as run_gaussian_exp.py:50-103 writes them."""
    lines = [f"base_lr: {base_lr}", f"momentum: {momentum}", f"weight_decay: {weight_decay}",
             f'lr_policy: "{lr_policy}"', f"max_iter: {max_iter}", f"test_iter: {test_iter}",
             f"test_interval: {test_interval}", f"display: {display}", f"random_seed: {random_seed}",
             f"test_initialization: {'true' if test_initialization else 'false'}"]
    for k, v in (("gamma", gamma), ("power", power), ("stepsize", stepsize), ("average_loss", average_loss)):
        if v is not None:
            lines.append(f"{k}: {v}")
    if failure_mean is not None:
        fp = f"failure_pattern {{ type: \"gaussian\" mean: {failure_mean} std: {failure_std}"
        if failure_prob is not None:
            neg, zero, pos = failure_prob
            fp += f" failure_prob {{ neg: {neg} zero: {zero} pos: {pos} }}"
        lines.append(fp + " }")
    if threshold is not None:
        lines.append(f'failure_strategy {{ type: "threshold" threshold: {threshold} }}')
    return "\n".join(lines) + "\n"


CONFIGS = {
    "lenet": (lenet, "1,28,28", 10),
    "cifar10_quick": (cifar10_quick, "3,32,32", 10),
    "cifar10_full": (cifar10_full, "3,32,32", 10),
    "alexnet": (alexnet, "3,256,256", 1000),
    "caffenet": (lambda **kw: alexnet(caffenet=True, **kw), "3,256,256", 1000),
    "googlenet": (googlenet, "3,256,256", 1000),
}


def net_options(name: str, **extra):
    _, shape, classes = CONFIGS[name]
    o = dict(data_shape=shape, num_classes=classes)
    o.update(extra)
    return o
