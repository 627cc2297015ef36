"""Golden layer tables of the configs' reference nets.

Run in the build container only (needs /root/reference and torch's bundled
protoc 3.13).  Parses each reference prototxt with protobuf's own text-format
parser over the reference schema, applies Caffe's phase rule (a layer runs in
a phase when it has no include rule matching another phase and no exclude rule
matching it; net.cpp FilterNet / StateMeetsRule, phase only) and writes
[name, type, bottoms, tops] per layer and phase to tests/golden/net_tables.json.
Nothing of the reference is committed beyond this table.

    python tests/golden/make_net_tables.py
"""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
REF = Path("/root/reference")
PROTOC = Path("/usr/local/lib/python3.10/dist-packages/torch/bin/protoc")
NETS = {
    "lenet": "examples/mnist/lenet_train_test.prototxt",
    "cifar10_quick": "examples/cifar10/cifar10_quick_train_test.prototxt",
    "cifar10_full": "examples/cifar10/cifar10_full_train_test.prototxt",
    "alexnet": "models/bvlc_alexnet/train_val.prototxt",
    "caffenet": "models/bvlc_reference_caffenet/train_val.prototxt",
    "googlenet": "models/bvlc_googlenet/train_val.prototxt",
}


def main():
    tmp = tempfile.mkdtemp()
    subprocess.check_call([str(PROTOC), f"-I{REF / 'src/caffe/proto'}", f"--python_out={tmp}",
                           str(REF / "src/caffe/proto/caffe.proto")])
    os.environ["PROTOCOL_BUFFERS_PYTHON_IMPLEMENTATION"] = "python"
    sys.path.insert(0, tmp)
    import caffe_pb2 as pb
    from google.protobuf import text_format

    def runs_in(layer, phase):
        if len(layer.include):
            return any((not r.HasField("phase")) or r.phase == phase for r in layer.include)
        return not any((not r.HasField("phase")) or r.phase == phase for r in layer.exclude)

    out = {}
    for key, rel in NETS.items():
        net = pb.NetParameter()
        text_format.Merge((REF / rel).read_text(), net)
        out[key] = {}
        for ph_name, ph in (("train", pb.TRAIN), ("test", pb.TEST)):
            out[key][ph_name] = [[l.name, l.type, list(l.bottom), list(l.top)] for l in net.layer if runs_in(l, ph)]
    (HERE / "net_tables.json").write_text(json.dumps(out, indent=0) + "\n")
    print("wrote", HERE / "net_tables.json", {k: len(v["test"]) for k, v in out.items()})


if __name__ == "__main__":
    main()
