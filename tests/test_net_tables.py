"""CPU tests of the prototxt path (no device): the configs' nets as this build
writes them (rramsim.models) and parses them (C++ text-format parser, phase
filter, split insertion: rram_net_describe) have the reference nets' layer
tables — names, types, bottoms and tops per phase — as protobuf parses the
reference prototxts (tests/golden/make_net_tables.py)."""
import json
from pathlib import Path

import pytest

GOLD = json.loads((Path(__file__).resolve().parent / "golden" / "net_tables.json").read_text())


def _unsplit(rows):
    """Undo Caffe's split insertion (insert_splits.cpp): drop Split layers and
    map split tops back to the blob they copy."""
    src = {}
    for name, typ, bots, tops in rows:
        if typ == "Split":
            for t in tops:
                src[t] = bots[0]
    return [[n, t, [src.get(b, b) for b in bots], tops] for n, t, bots, tops in rows if t != "Split"]


@pytest.mark.parametrize("key", ["lenet", "cifar10_quick", "cifar10_full", "alexnet", "caffenet", "googlenet"])
@pytest.mark.parametrize("phase", ["train", "test"])
def test_model_generators_match_reference_layer_tables(key, phase):
    from rramsim import caffe, models
    gen = models.alexnet(caffenet=True) if key == "caffenet" else getattr(models, key)()
    got = _unsplit(caffe.describe(gen, phase))
    exp = GOLD[key][phase]
    assert [r[:2] for r in got] == [r[:2] for r in exp]
    assert got == exp


def test_describe_inserts_splits_like_caffe():
    """A blob read by two layers gets a Split with Caffe's naming
    (insert_splits.cpp: <blob>_<layer>_<top>_split_<k>)."""
    from rramsim import caffe, models
    rows = caffe.describe(models.lenet(), "test")
    splits = [r for r in rows if r[1] == "Split"]
    assert splits, rows
    name, typ, bots, tops = splits[0]
    assert tops[0].startswith(bots[0] + "_") and tops[0].endswith("_split_0")
