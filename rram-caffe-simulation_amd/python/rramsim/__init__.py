"""rramsim — Python view of the MI355X-native RRAM fault-simulation path.

The product is two shared libraries built from rram-caffe-simulation_amd/:
  * librram_kernels.so — gfx950 HIP kernels behind the C-ABI include/rram_kernels.h
  * librram_caffe.so   — the C++ Caffe-shaped host (Blob/Layer/Net/Solver/
                         FailureMaker/Monte-Carlo driver) behind include/rram_caffe.h
This package only marshals arguments to them (ctypes); torch is used for device
memory, streams and torch.distributed.
"""
from . import _kernels as kernels  # noqa: F401
from ._kernels import (RramError, check, gaussian_fault_rate, make_inject_cfg,  # noqa: F401
                       mean_for_fault_rate, prob_threshold, split_thresholds)

__all__ = ["kernels", "RramError", "check", "gaussian_fault_rate", "make_inject_cfg",
           "mean_for_fault_rate", "prob_threshold", "split_thresholds"]
