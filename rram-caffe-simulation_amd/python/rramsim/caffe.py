"""ctypes view of the C++ host runtime (include/rram_caffe.h): Net, Solver,
MonteCarlo.  Mirrors pycaffe's shape of API (Net.forward/backward, blobs,
params; Solver.step/test) so tests read like the reference's own; every call
goes through librram_caffe.so -> librram_kernels.so.  No CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Optional

from . import _kernels as K

P, I, I64, U32, U64, F = C.c_void_p, C.c_int, C.c_int64, C.c_uint32, C.c_uint64, C.c_float
PP = C.POINTER(C.c_void_p)
PI = C.POINTER(C.c_int)
PI64 = C.POINTER(C.c_int64)
PF = C.POINTER(C.c_float)
CB = C.CFUNCTYPE(None, C.c_void_p)
LOGCB = C.CFUNCTYPE(None, C.c_char_p, C.c_void_p)
LAYERCB = C.CFUNCTYPE(None, C.c_int, C.c_void_p)

SIGNATURES = {
    "rram_caffe_last_error": (C.c_char_p, []),
    "rram_caffe_set_stream": (I, [P]),
    "rram_caffe_set_random_seed": (I, [U64]),
    "rram_caffe_synchronize": (I, []),
    "rram_net_create": (I, [C.c_char_p, I, C.c_char_p, PP]),
    "rram_net_destroy": (I, [P]),
    "rram_net_forward": (I, [P, I, PF]),
    "rram_net_backward": (I, [P]),
    "rram_net_update": (I, [P]),
    "rram_net_clear_param_diffs": (I, [P]),
    "rram_net_num_layers": (I, [P, PI]),
    "rram_net_layer_info": (I, [P, I, C.c_char_p, C.c_char_p, I, PI]),
    "rram_net_layer_contraction": (I, [P, I, C.POINTER(C.c_double), PI]),
    "rram_net_num_blobs": (I, [P, PI]),
    "rram_net_blob_name": (I, [P, I, C.c_char_p, I]),
    "rram_net_blob": (I, [P, C.c_char_p, PP, PP, PI, PI]),
    "rram_net_blob_stale": (I, [P, C.c_char_p, PI]),
    "rram_net_num_params": (I, [P, PI]),
    "rram_net_param": (I, [P, I, PP, PP, PI64, PF, PF]),
    "rram_net_num_failure_params": (I, [P, PI]),
    "rram_net_failure_param": (I, [P, I, PP, PP, PI64, PI]),
    "rram_net_num_outputs": (I, [P, PI]),
    "rram_net_output": (I, [P, I, C.c_char_p, I, PP, PI64]),
    "rram_net_share_trained": (I, [P, P]),
    "rram_net_flat_param_count": (I, [P, PI64]),
    "rram_net_alias_flat_params": (I, [P, P, P]),
    "rram_net_set_timing": (I, [P, I]),
    "rram_net_set_timing_layer": (I, [P, I]),
    "rram_net_layer_times": (I, [P, C.POINTER(C.c_double), C.POINTER(C.c_long), I, PI, I]),
    "rram_net_describe": (I, [C.c_char_p, I, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rram_mc_set_timing": (I, [P, I]),
    "rram_mc_set_reuse_prefix": (I, [P, I]),
    "rram_mc_set_graph": (I, [P, I]),
    "rram_mc_graph_active": (I, [P, PI]),
    "rram_mc_inject_times": (I, [P, C.POINTER(C.c_double), C.POINTER(C.c_long), PI64, I]),
    "rram_solver_create": (I, [C.c_char_p, C.c_char_p, C.c_char_p, PP]),
    "rram_solver_destroy": (I, [P]),
    "rram_solver_step": (I, [P, I]),
    "rram_solver_set_graph": (I, [P, I]),
    "rram_solver_graph_active": (I, [P, PI]),
    "rram_solver_solve": (I, [P]),
    "rram_solver_iter": (I, [P, PI]),
    "rram_solver_smoothed_loss": (I, [P, PF]),
    "rram_solver_learning_rate": (I, [P, PF]),
    "rram_solver_net": (I, [P, PP]),
    "rram_solver_num_test_nets": (I, [P, PI]),
    "rram_solver_test_net": (I, [P, I, PP]),
    "rram_solver_test": (I, [P, I, PF, I, PI]),
    "rram_solver_set_gradient_callback": (I, [P, CB, P]),
    "rram_solver_set_log_callback": (I, [P, LOGCB, P]),
    "rram_solver_set_backward_callback": (I, [P, LAYERCB, P]),
    "rram_solver_num_fail_blobs": (I, [P, PI]),
    "rram_solver_fail_state": (I, [P, I, PP, PP, PI64]),
    "rram_solver_broken_counts": (I, [P, C.POINTER(C.c_ulonglong), I, PI]),
    "rram_solver_num_history": (I, [P, PI]),
    "rram_solver_history": (I, [P, I, PP, PI64]),
    "rram_solver_apply_strategies": (I, [P]),
    "rram_solver_strategy_info": (I, [P, I, C.c_char_p, I, PI, PI, PI]),
    "rram_solver_snapshot": (I, [P, C.c_char_p, I]),
    "rram_solver_restore": (I, [P, C.c_char_p]),
    "rram_solver_solve_from": (I, [P, C.c_char_p]),
    "rram_net_copy_trained_layers_from": (I, [P, C.c_char_p]),
    "rram_net_save_weights": (I, [P, C.c_char_p, I]),
    "rram_caffemodel_describe": (I, [C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rram_proto_rewrite": (I, [C.c_char_p, C.c_char_p, I]),
    "rram_glibc_rand": (I, [U32, I, PI]),
    "rram_solver_describe": (I, [C.c_char_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "rram_syncedmem_create": (I, [C.c_size_t, PP]),
    "rram_syncedmem_destroy": (I, [P]),
    "rram_syncedmem_head": (I, [P, PI]),
    "rram_syncedmem_size": (I, [P, C.POINTER(C.c_size_t)]),
    "rram_syncedmem_cpu_data": (I, [P, PP]),
    "rram_syncedmem_gpu_data": (I, [P, PP]),
    "rram_syncedmem_mutable_cpu_data": (I, [P, PP]),
    "rram_syncedmem_mutable_gpu_data": (I, [P, PP]),
    "rram_syncedmem_set_cpu_data": (I, [P, P]),
    "rram_syncedmem_set_gpu_data": (I, [P, P]),
    "rram_mc_create": (I, [P, P, I, U64, I, PP]),
    "rram_mc_destroy": (I, [P]),
    "rram_mc_run": (I, [P, U32, U32]),
    "rram_mc_reset": (I, [P]),
    "rram_mc_restore_clean": (I, [P]),
    "rram_mc_stats": (I, [P, C.POINTER(C.c_double), I, PI, C.POINTER(C.c_ulonglong), I, PI, PF, I, PI]),
    "rram_comm_unique_id": (I, [C.c_char_p]),
    "rram_comm_create": (I, [C.c_char_p, I, I, PP]),
    "rram_comm_destroy": (I, [P]),
    "rram_comm_info": (I, [P, PI, PI]),
    "rram_comm_allreduce_f32": (I, [P, P, I64]),
    "rram_comm_allreduce_host_f64": (I, [P, C.POINTER(C.c_double), I, I]),
    "rram_comm_barrier": (I, [P]),
    "rram_dp_create": (I, [P, P, C.c_double, I, PP]),
    "rram_dp_destroy": (I, [P]),
    "rram_dp_info": (I, [P, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong), PI, PI64]),
    "rram_solver_flat_params": (I, [P, PP, PP, PI64]),
    "rram_mc_allreduce_stats": (I, [P, P, C.POINTER(C.c_double), I, PI]),
    "rram_dp_plan_buckets": (I, [I, PI, PI64, I64, PI, PI64, PI64, I, PI]),
}

_lib = None


def load():
    global _lib
    if _lib is None:
        K.load()  # kernels first (RTLD_GLOBAL)
        if not K.CAFFE_SO.exists():
            raise K.RramError(f"{K.CAFFE_SO} not built; there is no CPU fallback")
        lib = C.CDLL(str(K.CAFFE_SO))
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc, what=""):
    if rc != 0:
        raise K.RramError(f"{what} failed ({rc}): {load().rram_caffe_last_error().decode(errors='replace')}")


def set_stream_from_torch():
    import torch
    check(load().rram_caffe_set_stream(C.c_void_p(torch.cuda.current_stream().cuda_stream)), "set_stream")


def set_random_seed(seed: int):
    check(load().rram_caffe_set_random_seed(seed), "set_random_seed")


def synchronize():
    check(load().rram_caffe_synchronize(), "synchronize")


def options_text(opts: Optional[Dict]) -> Optional[bytes]:
    if not opts:
        return None
    parts = []
    for k, v in opts.items():
        if isinstance(v, bool):
            parts.append(f"{k}: {'true' if v else 'false'}")
        elif isinstance(v, (int, float)):
            parts.append(f"{k}: {v}")
        elif isinstance(v, (tuple, list)):
            parts.append(f'{k}: "{",".join(str(x) for x in v)}"')
        else:
            parts.append(f'{k}: "{v}"')
    return " ".join(parts).encode()


def describe(prototxt: str, phase: str = "test") -> List[tuple]:
    """Host-only structural view of a net (phase filter + split insertion):
    [(name, type, [bottoms], [tops])].  Needs no GPU."""
    lib = load()
    need = C.c_size_t()
    ph = 0 if phase == "train" else 1
    check(lib.rram_net_describe(prototxt.encode(), ph, None, 0, C.byref(need)), "net_describe")
    buf = C.create_string_buffer(need.value)
    check(lib.rram_net_describe(prototxt.encode(), ph, buf, need.value, None), "net_describe")
    out = []
    for line in buf.value.decode().splitlines():
        name, typ, bots, tops = line.split("\t")
        out.append((name, typ, [b for b in bots.split(",") if b], [t for t in tops.split(",") if t]))
    return out


def caffemodel_describe(path: str) -> List[tuple]:
    """Host-only: [(layer, type, blob_index, shape, count, data_sum, diff_count)]
    of a binary .caffemodel (NetParameter `layer` or V1 `layers`)."""
    lib = load()
    need = C.c_size_t()
    check(lib.rram_caffemodel_describe(str(path).encode(), None, 0, C.byref(need)), "caffemodel_describe")
    buf = C.create_string_buffer(need.value)
    check(lib.rram_caffemodel_describe(str(path).encode(), buf, need.value, None), "caffemodel_describe")
    out = []
    for line in buf.value.decode().splitlines():
        name, typ, idx, shape, n, dsum, ndiff = line.split("\t")
        out.append((name, typ, -1 if idx == "-" else int(idx), tuple(int(x) for x in shape.split(",") if x),
                    int(n), float(dsum), int(ndiff)))
    return out


def proto_rewrite(src: str, dst: str, kind: str = "net"):
    """Host-only: parse a binary proto and serialise it again (net | solverstate | blobs)."""
    k = {"net": 0, "solverstate": 1, "blobs": 2}[kind]
    check(load().rram_proto_rewrite(str(src).encode(), str(dst).encode(), k), "proto_rewrite")


def solver_describe(solver_prototxt: str) -> List[List[str]]:
    """Host-only: the failure_pattern / failure_strategy / solver key fields of
    a SolverParameter text as this build parses them (caffe.proto defaults applied)."""
    lib = load()
    need = C.c_size_t()
    check(lib.rram_solver_describe(solver_prototxt.encode(), None, 0, C.byref(need)), "solver_describe")
    buf = C.create_string_buffer(need.value)
    check(lib.rram_solver_describe(solver_prototxt.encode(), buf, need.value, None), "solver_describe")
    return [line.split("\t") for line in buf.value.decode().splitlines()]


def glibc_rand(seed: int, n: int) -> List[int]:
    """Host-only: n draws of the genetic strategy's glibc rand() after srand(seed)."""
    buf = (C.c_int * max(n, 1))()
    check(load().rram_glibc_rand(seed, n, buf), "glibc_rand")
    return [buf[i] for i in range(n)]


def _wrap_device(ptr: int, shape):
    """Zero-copy float32 torch view of a device pointer (via __cuda_array_interface__)."""
    import torch

    class _Iface:
        def __init__(self, p, s):
            self.__cuda_array_interface__ = {"shape": tuple(s), "typestr": "<f4", "data": (p, False),
                                             "version": 2, "strides": None}
    if len(shape) == 0:
        shape = (1,)
    return torch.as_tensor(_Iface(ptr, shape), device="cuda")


class SyncedMemory:
    """caffe::SyncedMemory (syncedmem.hpp:45-83): head() is one of
    UNINITIALIZED / HEAD_AT_CPU / HEAD_AT_GPU / SYNCED; the *_data calls
    return raw addresses (host or device) exactly like the C++ accessors."""
    UNINITIALIZED, HEAD_AT_CPU, HEAD_AT_GPU, SYNCED = range(4)

    def __init__(self, size: int):
        self._lib = load()
        h = C.c_void_p()
        check(self._lib.rram_syncedmem_create(size, C.byref(h)), "syncedmem_create")
        self.h = h

    def _ptr(self, fn) -> int:
        p = C.c_void_p()
        check(getattr(self._lib, fn)(self.h, C.byref(p)), fn)
        return p.value or 0

    def head(self) -> int:
        v = C.c_int()
        check(self._lib.rram_syncedmem_head(self.h, C.byref(v)), "syncedmem_head")
        return v.value

    def size(self) -> int:
        v = C.c_size_t()
        check(self._lib.rram_syncedmem_size(self.h, C.byref(v)), "syncedmem_size")
        return v.value

    def cpu_data(self) -> int:
        return self._ptr("rram_syncedmem_cpu_data")

    def gpu_data(self) -> int:
        return self._ptr("rram_syncedmem_gpu_data")

    def mutable_cpu_data(self) -> int:
        return self._ptr("rram_syncedmem_mutable_cpu_data")

    def mutable_gpu_data(self) -> int:
        return self._ptr("rram_syncedmem_mutable_gpu_data")

    def set_cpu_data(self, addr: int):
        check(self._lib.rram_syncedmem_set_cpu_data(self.h, C.c_void_p(addr)), "syncedmem_set_cpu_data")

    def set_gpu_data(self, addr: int):
        check(self._lib.rram_syncedmem_set_gpu_data(self.h, C.c_void_p(addr)), "syncedmem_set_gpu_data")

    def close(self):
        if getattr(self, "h", None):
            self._lib.rram_syncedmem_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Net:
    """caffe::Net<float> (net.cpp).  phase: 'train' | 'test'."""

    def __init__(self, prototxt: str, phase: str = "test", options: Optional[Dict] = None,
                 _handle=None, _owned=True):
        self._lib = load()
        if _handle is not None:
            self.h = _handle
        else:
            h = C.c_void_p()
            check(self._lib.rram_net_create(prototxt.encode(), 0 if phase == "train" else 1,
                                            options_text(options), C.byref(h)), "net_create")
            self.h = h
        self._owned = _owned and _handle is None

    def close(self):
        if getattr(self, "_owned", False) and self.h:
            self._lib.rram_net_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def forward(self, compute_loss=True) -> float:
        loss = C.c_float(0)
        check(self._lib.rram_net_forward(self.h, int(compute_loss), C.byref(loss)), "forward")
        return loss.value

    def backward(self):
        check(self._lib.rram_net_backward(self.h), "backward")

    def update(self):
        check(self._lib.rram_net_update(self.h), "update")

    def clear_param_diffs(self):
        check(self._lib.rram_net_clear_param_diffs(self.h), "clear_param_diffs")

    def layers(self) -> List[tuple]:
        n = C.c_int()
        check(self._lib.rram_net_num_layers(self.h, C.byref(n)), "num_layers")
        out = []
        for i in range(n.value):
            name, typ, np_ = C.create_string_buffer(256), C.create_string_buffer(256), C.c_int()
            check(self._lib.rram_net_layer_info(self.h, i, name, typ, 256, C.byref(np_)), "layer_info")
            out.append((name.value.decode(), typ.value.decode(), np_.value))
        return out

    def contractions(self) -> Dict[str, tuple]:
        """{layer name: (forward FLOPs, engine)} for the Convolution and
        InnerProduct layers at the current shapes (rram_net_layer_contraction;
        engine 0 = fp32 MFMA, 1 = bf16x6)."""
        out = {}
        for i, (name, typ, _) in enumerate(self.layers()):
            f, e = C.c_double(), C.c_int()
            check(self._lib.rram_net_layer_contraction(self.h, i, C.byref(f), C.byref(e)), "layer_contraction")
            if e.value >= 0:
                out[name] = (f.value, e.value)
        return out

    def blob_names(self) -> List[str]:
        n = C.c_int()
        check(self._lib.rram_net_num_blobs(self.h, C.byref(n)), "num_blobs")
        names = []
        for i in range(n.value):
            b = C.create_string_buffer(512)
            check(self._lib.rram_net_blob_name(self.h, i, b, 512), "blob_name")
            names.append(b.value.decode())
        return names

    def blob(self, name: str, diff=False):
        d, g = C.c_void_p(), C.c_void_p()
        shape = (C.c_int * 8)()
        na = C.c_int()
        # ask only for the pointer wanted: a data read materialises folded
        # blobs (rram_net_blob), a diff read must not undo the folds
        check(self._lib.rram_net_blob(self.h, name.encode(), None if diff else C.byref(d),
                                      C.byref(g) if diff else None, shape, C.byref(na)),
              f"blob {name}")
        return _wrap_device((g if diff else d).value, [shape[i] for i in range(na.value)])

    def blob_stale(self, name: str) -> bool:
        """True when the last forward left the blob's fp32 contents unwritten
        (the pooled-output fold); blob() materialises it."""
        st = C.c_int()
        check(self._lib.rram_net_blob_stale(self.h, name.encode(), C.byref(st)), f"blob_stale {name}")
        return bool(st.value)

    def params(self):
        n = C.c_int()
        check(self._lib.rram_net_num_params(self.h, C.byref(n)), "num_params")
        out = []
        for i in range(n.value):
            d, g, cnt, lr, dm = C.c_void_p(), C.c_void_p(), C.c_int64(), C.c_float(), C.c_float()
            check(self._lib.rram_net_param(self.h, i, C.byref(d), C.byref(g), C.byref(cnt), C.byref(lr),
                                           C.byref(dm)), "param")
            out.append(dict(data=_wrap_device(d.value, (cnt.value,)), diff=_wrap_device(g.value, (cnt.value,)),
                            lr_mult=lr.value, decay_mult=dm.value))
        return out

    def failure_params(self):
        n = C.c_int()
        check(self._lib.rram_net_num_failure_params(self.h, C.byref(n)), "num_failure_params")
        out = []
        for i in range(n.value):
            d, g, cnt, lid = C.c_void_p(), C.c_void_p(), C.c_int64(), C.c_int()
            check(self._lib.rram_net_failure_param(self.h, i, C.byref(d), C.byref(g), C.byref(cnt),
                                                   C.byref(lid)), "failure_param")
            out.append(dict(data=_wrap_device(d.value, (cnt.value,)), diff=_wrap_device(g.value, (cnt.value,)),
                            count=cnt.value, layer_id=lid.value))
        return out

    def outputs(self) -> Dict[str, object]:
        n = C.c_int()
        check(self._lib.rram_net_num_outputs(self.h, C.byref(n)), "num_outputs")
        out = {}
        for i in range(n.value):
            name, d, cnt = C.create_string_buffer(256), C.c_void_p(), C.c_int64()
            check(self._lib.rram_net_output(self.h, i, name, 256, C.byref(d), C.byref(cnt)), "output")
            out[name.value.decode()] = _wrap_device(d.value, (cnt.value,))
        return out

    def set_timing(self, mode):
        """False/0 off, True/1 every layer, 2 only parameter layers (conv / IP)."""
        check(self._lib.rram_net_set_timing(self.h, int(mode)), "set_timing")

    def set_timing_layer(self, name):
        """hipEvents around the named layer only."""
        idx = [i for i, (nm, _, _) in enumerate(self.layers()) if nm == name]
        if not idx:
            raise KeyError(name)
        check(self._lib.rram_net_set_timing_layer(self.h, idx[0]), "set_timing_layer")

    def layer_times(self, reset=False):
        """[(layer name, type, total ms, launches)] since the last reset."""
        L = self.layers()
        ms = (C.c_double * len(L))()
        cnt = (C.c_long * len(L))()
        n = C.c_int()
        check(self._lib.rram_net_layer_times(self.h, ms, cnt, len(L), C.byref(n), int(reset)), "layer_times")
        return [(L[i][0], L[i][1], ms[i], cnt[i]) for i in range(len(L))]

    def share_trained_with(self, other: "Net"):
        check(self._lib.rram_net_share_trained(self.h, other.h), "share_trained")

    def copy_from(self, caffemodel: str):
        """Net::CopyTrainedLayersFrom (binary .caffemodel)."""
        check(self._lib.rram_net_copy_trained_layers_from(self.h, str(caffemodel).encode()), "copy_trained_layers_from")

    def save(self, caffemodel: str, write_diff: bool = False):
        """Net::ToProto + WriteProtoToBinaryFile."""
        check(self._lib.rram_net_save_weights(self.h, str(caffemodel).encode(), int(write_diff)), "save_weights")

    def flat_param_count(self) -> int:
        n = C.c_int64()
        check(self._lib.rram_net_flat_param_count(self.h, C.byref(n)), "flat_param_count")
        return n.value

    def alias_flat_params(self, data_t, diff_t):
        check(self._lib.rram_net_alias_flat_params(self.h, C.c_void_p(data_t.data_ptr()),
                                                   C.c_void_p(diff_t.data_ptr())), "alias_flat_params")


class Solver:
    """caffe::SGDSolver with the fork's fault hooks."""

    def __init__(self, solver_prototxt: str, net_prototxt: Optional[str] = None,
                 options: Optional[Dict] = None, log=None):
        self._lib = load()
        h = C.c_void_p()
        check(self._lib.rram_solver_create(solver_prototxt.encode(),
                                           net_prototxt.encode() if net_prototxt else None,
                                           options_text(options), C.byref(h)), "solver_create")
        self.h = h
        self._cb = None
        self._logcb = None
        self.log_lines: List[str] = []

        def _log(line, _user):
            s = line.decode()
            self.log_lines.append(s)
            if log:
                log(s)
        self._logcb = LOGCB(_log)
        check(self._lib.rram_solver_set_log_callback(self.h, self._logcb, None), "set_log_callback")

    def close(self):
        if self.h:
            self._lib.rram_solver_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def net(self) -> Net:
        n = C.c_void_p()
        check(self._lib.rram_solver_net(self.h, C.byref(n)), "solver_net")
        return Net("", _handle=n, _owned=False)

    def test_net(self, i=0) -> Net:
        n = C.c_void_p()
        check(self._lib.rram_solver_test_net(self.h, i, C.byref(n)), "solver_test_net")
        return Net("", _handle=n, _owned=False)

    @property
    def iter(self) -> int:
        v = C.c_int()
        check(self._lib.rram_solver_iter(self.h, C.byref(v)), "iter")
        return v.value

    def learning_rate(self) -> float:
        v = C.c_float()
        check(self._lib.rram_solver_learning_rate(self.h, C.byref(v)), "learning_rate")
        return v.value

    def smoothed_loss(self) -> float:
        v = C.c_float()
        check(self._lib.rram_solver_smoothed_loss(self.h, C.byref(v)), "smoothed_loss")
        return v.value

    def set_graph(self, on: bool):
        """Opt-in hipGraph replay of the training iteration (include/rram_caffe.h rram_solver_set_graph)."""
        check(self._lib.rram_solver_set_graph(self.h, int(on)), "solver_set_graph")

    def graph_active(self) -> bool:
        a = C.c_int()
        check(self._lib.rram_solver_graph_active(self.h, C.byref(a)), "solver_graph_active")
        return bool(a.value)

    def step(self, iters: int):
        check(self._lib.rram_solver_step(self.h, iters), "step")

    def solve(self, resume_file: Optional[str] = None):
        if resume_file is None:
            check(self._lib.rram_solver_solve(self.h), "solve")
        else:
            check(self._lib.rram_solver_solve_from(self.h, str(resume_file).encode()), "solve")

    def snapshot(self) -> str:
        buf = C.create_string_buffer(4096)
        check(self._lib.rram_solver_snapshot(self.h, buf, 4096), "snapshot")
        return buf.value.decode()

    def restore(self, state_file: str):
        check(self._lib.rram_solver_restore(self.h, str(state_file).encode()), "restore")

    def apply_strategies(self):
        check(self._lib.rram_solver_apply_strategies(self.h), "apply_strategies")

    def strategy_info(self, i=0):
        t = C.create_string_buffer(64)
        a, b, c = C.c_int(), C.c_int(), C.c_int()
        check(self._lib.rram_solver_strategy_info(self.h, i, t, 64, C.byref(a), C.byref(b), C.byref(c)),
              "strategy_info")
        return t.value.decode(), a.value, b.value, c.value

    def test(self, i=0) -> List[float]:
        buf = (C.c_float * 1024)()
        n = C.c_int()
        check(self._lib.rram_solver_test(self.h, i, buf, 1024, C.byref(n)), "test")
        return [buf[k] for k in range(n.value)]

    def flat_params(self):
        """(data, diff) device views of the solver's flat learnable buffers
        (every param aliased into them, the GPUParams layout), or None."""
        d, g, n = C.c_void_p(), C.c_void_p(), C.c_int64()
        check(self._lib.rram_solver_flat_params(self.h, C.byref(d), C.byref(g), C.byref(n)), "solver_flat_params")
        if not d.value:
            return None
        return _wrap_device(d.value, (n.value,)), _wrap_device(g.value, (n.value,))

    def set_gradient_callback(self, fn):
        self._cb = CB(lambda _u: fn())
        check(self._lib.rram_solver_set_gradient_callback(self.h, self._cb, None), "set_gradient_callback")

    def set_backward_callback(self, fn):
        """fn(layer_index) after each train-net layer's Backward (None = off)."""
        if fn is None:
            self._bwdcb = None
            check(self._lib.rram_solver_set_backward_callback(self.h, LAYERCB(), None), "set_backward_callback")
            return
        self._bwdcb = LAYERCB(lambda i, _u: fn(i))
        check(self._lib.rram_solver_set_backward_callback(self.h, self._bwdcb, None), "set_backward_callback")

    def fail_state(self):
        n = C.c_int()
        check(self._lib.rram_solver_num_fail_blobs(self.h, C.byref(n)), "num_fail_blobs")
        out = []
        for i in range(n.value):
            e, v, cnt = C.c_void_p(), C.c_void_p(), C.c_int64()
            check(self._lib.rram_solver_fail_state(self.h, i, C.byref(e), C.byref(v), C.byref(cnt)), "fail_state")
            out.append((_wrap_device(e.value, (cnt.value,)), _wrap_device(v.value, (cnt.value,))))
        return out

    def broken_counts(self) -> List[int]:
        buf = (C.c_ulonglong * 256)()
        n = C.c_int()
        check(self._lib.rram_solver_broken_counts(self.h, buf, 256, C.byref(n)), "broken_counts")
        return [buf[i] for i in range(n.value)]

    def history(self):
        """SGDSolver::history(): momentum blob per learnable param (device views)."""
        n = C.c_int()
        check(self._lib.rram_solver_num_history(self.h, C.byref(n)), "num_history")
        out = []
        for i in range(n.value):
            d, cnt = C.c_void_p(), C.c_int64()
            check(self._lib.rram_solver_history(self.h, i, C.byref(d), C.byref(cnt)), "history")
            out.append(_wrap_device(d.value, (cnt.value,)))
        return out


class MonteCarlo:
    """Fault-map Monte-Carlo inference driver (rram_mc_*)."""

    def __init__(self, net: Net, cfgs, seed: int, max_maps: int = 4096):
        self._lib = load()
        if not isinstance(cfgs, (list, tuple)):
            cfgs = [cfgs]
        arr = (K.InjectCfg * len(cfgs))(*cfgs)
        h = C.c_void_p()
        check(self._lib.rram_mc_create(net.h, C.cast(arr, C.c_void_p), len(cfgs), seed, max_maps, C.byref(h)),
              "mc_create")
        self.h, self.net, self.max_maps = h, net, max_maps

    def run(self, begin: int, count: int):
        check(self._lib.rram_mc_run(self.h, begin, count), "mc_run")

    def reset(self):
        check(self._lib.rram_mc_reset(self.h), "mc_reset")

    def restore_clean(self):
        check(self._lib.rram_mc_restore_clean(self.h), "mc_restore_clean")

    def set_timing(self, on: bool):
        check(self._lib.rram_mc_set_timing(self.h, int(on)), "mc_set_timing")

    def set_reuse_prefix(self, on: bool):
        """Opt-in: run the layers before the first faultable one once for a
        fixed input batch (include/rram_caffe.h rram_mc_set_reuse_prefix)."""
        check(self._lib.rram_mc_set_reuse_prefix(self.h, int(on)), "mc_set_reuse_prefix")

    def set_graph(self, on: bool):
        """Opt-in hipGraph replay of the maps (include/rram_caffe.h rram_mc_set_graph)."""
        check(self._lib.rram_mc_set_graph(self.h, int(on)), "mc_set_graph")

    def graph_active(self) -> bool:
        a = C.c_int()
        check(self._lib.rram_mc_graph_active(self.h, C.byref(a)), "mc_graph_active")
        return bool(a.value)

    def inject_times(self, reset=False):
        """(total ms, launches, faultable weights) of the injection launches."""
        ms, n, w = C.c_double(), C.c_long(), C.c_int64()
        check(self._lib.rram_mc_inject_times(self.h, C.byref(ms), C.byref(n), C.byref(w), int(reset)),
              "mc_inject_times")
        return ms.value, n.value, w.value

    def stats(self):
        sums = (C.c_double * 64)()
        broken = (C.c_ulonglong * 256)()
        per_map = (C.c_float * (self.max_maps * 8))()
        no, nb, mr = C.c_int(), C.c_int(), C.c_int()
        check(self._lib.rram_mc_stats(self.h, sums, 64, C.byref(no), broken, 256, C.byref(nb), per_map,
                                      self.max_maps * 8, C.byref(mr)), "mc_stats")
        n_out = no.value
        pm = [[per_map[m * n_out + k] for k in range(n_out)] for m in range(min(mr.value, self.max_maps))]
        return dict(sums=[sums[i] for i in range(n_out)], broken=[broken[i] for i in range(nb.value)],
                    per_map=pm, maps=mr.value)

    def summary(self, z: float = 1.96):
        """Per-output statistics over the maps run: mean, sample
        std and the normal-approximation confidence half-width z*std/sqrt(n) from
        the per-map records, plus the mean broken cells per faultable blob."""
        st = self.stats()
        names = [k for k, v in self.net.outputs().items() if v.numel() == 1]
        pm = st["per_map"]
        n = len(pm)
        out = {}
        for k, name in enumerate(names[:len(st["sums"])]):
            vals = [row[k] for row in pm]
            mean = st["sums"][k] / max(st["maps"], 1)
            std = (sum((v - sum(vals) / n) ** 2 for v in vals) / (n - 1)) ** 0.5 if n > 1 else 0.0
            out[name] = dict(mean=mean, std=std, ci=z * std / n ** 0.5 if n > 1 else float("inf"), maps=st["maps"])
        out["_broken_per_map"] = [b / max(st["maps"], 1) for b in st["broken"]]
        return out

    def log_lines(self, iteration: int = 0) -> List[str]:
        """The reference's Solver::Test lines (solver.cpp:440-456) for the map
        means, which examples/cifar10/plot_pic.py and tools/extra/parse_log.py read."""
        s = self.summary()
        lines = [f"Iteration {iteration}, Testing net (#0)"]
        for k, (name, v) in enumerate((n, v) for n, v in s.items() if not n.startswith("_")):
            lines.append(f"    Test net output #{k}: {name} = {v['mean']:g}")
        return lines

    def close(self):
        if self.h:
            self._lib.rram_mc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Comm:
    """RCCL communicator of the C++ host (include/rram_caffe.h rram_comm_*):
    the collective the native P2PSync (rram_dp_*) and the Monte-Carlo stats
    reduction run on.  Rank 0 draws the 128-byte id; with world > 1 it reaches
    the other ranks through torch.distributed's rendezvous (plumbing only:
    broadcast_object_list on the process group, any backend), after which
    every collective is RCCL called from librram_caffe.so."""

    def __init__(self, rank: int = 0, world: int = 1, group=None):
        self._lib = load()
        uid = C.create_string_buffer(128)
        if rank == 0:
            check(self._lib.rram_comm_unique_id(uid), "comm_unique_id")
        if world > 1:
            import torch.distributed as dist
            box = [uid.raw if rank == 0 else None]
            dist.broadcast_object_list(box, src=0, group=group)
            uid = C.create_string_buffer(box[0], 128)
        h = C.c_void_p()
        check(self._lib.rram_comm_create(uid, rank, world, C.byref(h)), "comm_create")
        self.h, self.rank, self.world = h, rank, world

    def allreduce_host(self, vals, op: str = "sum") -> List[float]:
        """All-reduce of host doubles (sum | max), synchronous."""
        buf = (C.c_double * max(len(vals), 1))(*vals)
        check(self._lib.rram_comm_allreduce_host_f64(self.h, buf, len(vals), {"sum": 0, "max": 1}[op]),
              "comm_allreduce_host_f64")
        return [buf[i] for i in range(len(vals))]

    def allreduce_(self, t):
        """In-place sum all-reduce of a contiguous float32 device tensor on the
        host runtime's stream (asynchronous)."""
        assert t.dtype.is_floating_point and t.element_size() == 4 and t.is_contiguous()
        check(self._lib.rram_comm_allreduce_f32(self.h, C.c_void_p(t.data_ptr()), t.numel()), "comm_allreduce_f32")

    def barrier(self):
        check(self._lib.rram_comm_barrier(self.h), "comm_barrier")

    def mc_stats(self, mc: "MonteCarlo") -> List[float]:
        """MonteCarlo statistics summed over every rank: output sums, broken
        cells, maps (rram_mc_allreduce_stats, one RCCL all-reduce)."""
        buf = (C.c_double * 64)()
        n = C.c_int()
        check(self._lib.rram_mc_allreduce_stats(mc.h, self.h, buf, 64, C.byref(n)), "mc_allreduce_stats")
        return [buf[i] for i in range(n.value)]

    def close(self):
        if self.h:
            self._lib.rram_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def dp_plan_buckets(layer_ranges, bucket_elems: int) -> Dict[int, tuple]:
    """Host-only: the C++ P2PSync's bucket plan (rram_dp_plan_buckets) in the
    form of rramsim.parallel.plan_buckets: {layer: (begin, end)}."""
    nr = (C.c_int * max(len(layer_ranges), 1))(*[len(r) for r in layer_ranges])
    flat = [x for r in layer_ranges for pair in r for x in pair]
    rr = (C.c_int64 * max(len(flat), 1))(*flat)
    cap = max(len(layer_ranges), 1)
    lay, lo, hi, n = (C.c_int * cap)(), (C.c_int64 * cap)(), (C.c_int64 * cap)(), C.c_int()
    check(load().rram_dp_plan_buckets(len(layer_ranges), nr, rr, bucket_elems, lay, lo, hi, cap, C.byref(n)),
          "dp_plan_buckets")
    return {lay[k]: (lo[k], hi[k]) for k in range(n.value)}


class P2PSync:
    """The native data-parallel hooks (rram_dp_*): parameter broadcast from
    rank 0 now, then per iteration the RCCL all-reduce of the flat gradient
    buffer + 1/N inside the solver's step (bucketed on a collective stream
    when overlap is on)."""

    def __init__(self, solver: Solver, comm: Comm, bucket_mb: float = 4.0, overlap: bool = False):
        self._lib = load()
        h = C.c_void_p()
        check(self._lib.rram_dp_create(solver.h, comm.h, float(bucket_mb), int(overlap), C.byref(h)), "dp_create")
        self.h, self.solver, self.comm = h, solver, comm

    def info(self):
        a, b, nb, n = C.c_longlong(), C.c_longlong(), C.c_int(), C.c_int64()
        check(self._lib.rram_dp_info(self.h, C.byref(a), C.byref(b), C.byref(nb), C.byref(n)), "dp_info")
        return dict(allreduce_calls=a.value, bucket_calls=b.value, buckets=nb.value, params=n.value)

    def close(self):
        if self.h:
            self._lib.rram_dp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
