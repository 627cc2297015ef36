"""SyncedMemory head-state machine, mirroring the
reference's src/caffe/test/test_syncedmem.cpp:15-125 through the C-ABI
(include/rram_caffe.h rram_syncedmem_*).  The host-only transitions run on the
CPU; every transition that touches the device is a `gpu` test."""
import ctypes

import pytest

# --------------------------------------------------------------- host only


def _sm():
    from rramsim.caffe import SyncedMemory
    return SyncedMemory


def test_initialization():                                   # test_syncedmem.cpp:15-22
    SM = _sm()
    m = SM(10)
    assert m.head() == SM.UNINITIALIZED and m.size() == 10
    m2 = SM(10 * 4)
    assert m2.size() == 40
    m.close()
    m2.close()


def test_allocation_cpu():                                   # :38-42
    SM = _sm()
    m = SM(10)
    assert m.cpu_data() and m.mutable_cpu_data()
    m.close()


def test_cpu_write():                                        # :54-69
    SM = _sm()
    m = SM(10)
    p = m.mutable_cpu_data()
    assert m.head() == SM.HEAD_AT_CPU
    ctypes.memset(p, 1, m.size())
    assert ctypes.string_at(p, 10) == b"\x01" * 10
    p = m.mutable_cpu_data()                                 # another round
    assert m.head() == SM.HEAD_AT_CPU
    ctypes.memset(p, 2, m.size())
    assert ctypes.string_at(m.cpu_data(), 10) == b"\x02" * 10
    m.close()


def test_fresh_cpu_data_is_zeroed_and_const_read_keeps_head():
    SM = _sm()
    m = SM(64)
    p = m.cpu_data()                                         # UNINITIALIZED -> HEAD_AT_CPU (calloc)
    assert m.head() == SM.HEAD_AT_CPU and ctypes.string_at(p, 64) == b"\x00" * 64
    assert m.cpu_data() == p and m.head() == SM.HEAD_AT_CPU
    m.close()


def test_set_cpu_data_borrows_without_free():                # syncedmem.cpp:84-94
    SM = _sm()
    buf = ctypes.create_string_buffer(b"\x07" * 16, 16)
    m = SM(16)
    m.mutable_cpu_data()
    m.set_cpu_data(ctypes.addressof(buf))
    assert m.head() == SM.HEAD_AT_CPU and m.cpu_data() == ctypes.addressof(buf)
    m.close()                                                # must not free the borrowed buffer
    assert buf.raw == b"\x07" * 16


def test_null_borrow_is_an_error_not_an_abort():
    from rramsim import RramError
    SM = _sm()
    m = SM(8)
    with pytest.raises(RramError, match="set_cpu_data"):
        m.set_cpu_data(0)
    m.close()


# ------------------------------------------------------------------ device
@pytest.mark.gpu
def test_allocation_cpu_gpu(device):                         # :26-32, :46-50
    SM = _sm()
    m = SM(10)
    assert m.cpu_data() and m.gpu_data() and m.mutable_cpu_data() and m.mutable_gpu_data()
    m.close()
    g = SM(10)
    assert g.gpu_data() and g.mutable_gpu_data()
    g.close()


def _d2h(addr, n):
    import torch
    from rramsim.caffe import _wrap_device
    torch.cuda.synchronize()
    t = _wrap_device(addr, (n // 4,))
    return t.cpu().numpy().tobytes()


def _dmemset(addr, byte, n):
    import torch
    from rramsim.caffe import _wrap_device
    t = _wrap_device(addr, (n // 4,))
    t.view(torch.uint8).fill_(byte)
    torch.cuda.synchronize()


@pytest.mark.gpu
def test_gpu_read(device):                                   # :75-103
    from rramsim import caffe
    caffe.set_stream_from_torch()
    SM = _sm()
    m = SM(16)
    p = m.mutable_cpu_data()
    assert m.head() == SM.HEAD_AT_CPU
    ctypes.memset(p, 1, 16)
    g = m.gpu_data()
    assert m.head() == SM.SYNCED and _d2h(g, 16) == b"\x01" * 16
    p = m.mutable_cpu_data()                                 # another round
    assert m.head() == SM.HEAD_AT_CPU
    ctypes.memset(p, 2, 16)
    g2 = m.gpu_data()
    assert g2 == g                                           # the device buffer is reused
    assert m.head() == SM.SYNCED and _d2h(g2, 16) == b"\x02" * 16
    m.close()


@pytest.mark.gpu
def test_gpu_write(device):                                  # :105-123
    from rramsim import caffe
    caffe.set_stream_from_torch()
    SM = _sm()
    m = SM(16)
    g = m.mutable_gpu_data()
    assert m.head() == SM.HEAD_AT_GPU
    assert _d2h(g, 16) == b"\x00" * 16                       # fresh device memory is zeroed
    _dmemset(g, 1, 16)
    c = m.cpu_data()
    assert ctypes.string_at(c, 16) == b"\x01" * 16 and m.head() == SM.SYNCED
    g = m.mutable_gpu_data()
    assert m.head() == SM.HEAD_AT_GPU
    _dmemset(g, 2, 16)
    c2 = m.cpu_data()
    assert c2 == c and ctypes.string_at(c2, 16) == b"\x02" * 16 and m.head() == SM.SYNCED
    m.close()


@pytest.mark.gpu
def test_full_walk_and_set_gpu_data_borrow(device):
    """UNINITIALIZED -> HEAD_AT_CPU -> SYNCED -> HEAD_AT_GPU -> SYNCED ->
    HEAD_AT_CPU, data checked at every step; then set_gpu_data (the P2PSync /
    flat-buffer aliasing path, syncedmem.cpp:104-122) borrows a torch tensor:
    head HEAD_AT_GPU, reads come from it, and destroying the SyncedMemory leaves
    the borrowed buffer alive and unchanged."""
    import numpy as np
    import torch
    from rramsim import caffe
    caffe.set_stream_from_torch()
    SM = _sm()
    n = 4096
    m = SM(n)
    assert m.head() == SM.UNINITIALIZED
    c = m.mutable_cpu_data()
    ctypes.memmove(c, np.arange(n // 4, dtype=np.float32).tobytes(), n)
    assert m.head() == SM.HEAD_AT_CPU
    g = m.gpu_data()
    assert m.head() == SM.SYNCED
    assert np.array_equal(np.frombuffer(_d2h(g, n), np.float32), np.arange(n // 4, dtype=np.float32))
    g = m.mutable_gpu_data()
    assert m.head() == SM.HEAD_AT_GPU
    _dmemset(g, 0x3F, n)
    m.cpu_data()
    assert m.head() == SM.SYNCED and ctypes.string_at(m.cpu_data(), n) == b"\x3f" * n
    m.mutable_cpu_data()
    assert m.head() == SM.HEAD_AT_CPU
    # borrow external device memory
    ext = torch.full((n // 4,), 3.5, device=device)
    m.set_gpu_data(ext.data_ptr())
    assert m.head() == SM.HEAD_AT_GPU and m.gpu_data() == ext.data_ptr()
    assert np.all(np.frombuffer(ctypes.string_at(m.cpu_data(), n), np.float32) == 3.5)
    assert m.head() == SM.SYNCED
    m.close()
    torch.cuda.synchronize()
    assert torch.all(ext == 3.5)                             # not freed, not modified
    ext.add_(1.0)
    torch.cuda.synchronize()
    assert torch.all(ext == 4.5)
