"""Generate the binary-proto fixtures with
protobuf's own serializer over the reference schema.

Run in the build container only (needs /root/reference and torch's bundled
protoc 3.13; nothing generated from the reference is committed, only the
small binary fixtures and their expected descriptions):

    python tests/golden/make_proto_golden.py

Outputs (tests/golden/):
  tiny_net.caffemodel     NetParameter, `layer` (V2) with InnerProduct blobs
                          (shape + data, one blob with diff), a blob-less ReLU
  tiny_v1.caffemodel      NetParameter, V1 `layers` with legacy 4-D blob dims
                          and INNER_PRODUCT type enum
  tiny.solverstate        SolverState (iter, learned_net, history, current_step)
  proto_golden.json       the expected per-blob descriptions
"""
import json
import os
import subprocess
import sys
import tempfile
from pathlib import Path

HERE = Path(__file__).resolve().parent
PROTO_DIR = Path("/root/reference/src/caffe/proto")
PROTOC = Path("/usr/local/lib/python3.10/dist-packages/torch/bin/protoc")


def vals(n, seed):
    # exactly representable fp32 values (k/64), deterministic
    return [((i * 37 + seed * 11) % 257 - 128) / 64.0 for i in range(n)]


def main():
    tmp = tempfile.mkdtemp()
    subprocess.check_call([str(PROTOC), f"-I{PROTO_DIR}", f"--python_out={tmp}", str(PROTO_DIR / "caffe.proto")])
    os.environ["PROTOCOL_BUFFERS_PYTHON_IMPLEMENTATION"] = "python"
    sys.path.insert(0, tmp)
    import caffe_pb2 as pb

    expect = {}
    # ---- V2 net
    net = pb.NetParameter()
    net.name = "tiny"
    spec = [("ip1", "InnerProduct", ["data"], ["ip1"], [(3, 4), (3,)]),
            ("relu1", "ReLU", ["ip1"], ["ip1"], []),
            ("ip2", "InnerProduct", ["ip1"], ["ip2"], [(2, 3), (2,)])]
    rows = []
    for li, (name, typ, bot, top, shapes) in enumerate(spec):
        L = net.layer.add()
        L.name, L.type = name, typ
        L.bottom.extend(bot)
        L.top.extend(top)
        for j, sh in enumerate(shapes):
            b = L.blobs.add()
            b.shape.dim.extend(sh)
            n = 1
            for d in sh:
                n *= d
            v = vals(n, 10 * li + j)
            b.data.extend(v)
            nd = 0
            if name == "ip2" and j == 0:
                b.diff.extend(vals(n, 99))
                nd = n
            rows.append([name, typ, j, list(sh), n, sum(v), nd])
        if not shapes:
            rows.append([name, typ, -1, [], 0, 0.0, 0])
    (HERE / "tiny_net.caffemodel").write_bytes(net.SerializeToString())
    expect["tiny_net"] = rows

    # ---- V1 net (legacy dims)
    v1 = pb.NetParameter()
    v1.name = "tiny_v1"
    rows = []
    L = v1.layers.add()
    L.name = "fc"
    L.type = pb.V1LayerParameter.INNER_PRODUCT
    L.bottom.append("data")
    L.top.append("fc")
    for j, (num, ch, h, w) in enumerate([(1, 1, 2, 5), (1, 1, 1, 2)]):
        b = L.blobs.add()
        b.num, b.channels, b.height, b.width = num, ch, h, w
        n = num * ch * h * w
        v = vals(n, 50 + j)
        b.data.extend(v)
        rows.append(["fc", "InnerProduct", j, [num, ch, h, w], n, sum(v), 0])
    (HERE / "tiny_v1.caffemodel").write_bytes(v1.SerializeToString())
    expect["tiny_v1"] = rows

    # ---- SolverState
    st = pb.SolverState()
    st.iter = 7
    st.learned_net = "snap_iter_7.caffemodel"
    st.current_step = 1
    for j, sh in enumerate([(3, 4), (3,)]):
        b = st.history.add()
        b.shape.dim.extend(sh)
        n = 1
        for d in sh:
            n *= d
        b.data.extend(vals(n, 70 + j))
    (HERE / "tiny.solverstate").write_bytes(st.SerializeToString())
    expect["tiny_solverstate"] = {"iter": 7, "learned_net": st.learned_net, "current_step": 1,
                                  "history_counts": [12, 3]}
    (HERE / "proto_golden.json").write_text(json.dumps(expect, indent=1) + "\n")
    print("wrote", sorted(p.name for p in HERE.glob("tiny*")))


if __name__ == "__main__":
    main()
