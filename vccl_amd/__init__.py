"""vccl_amd — MI355X-native bucket-reduction path of VCCL (reduce-copy + ring
all-reduce / reduce-scatter / all-gather over xGMI), behind the reference's
ncclAllReduce / ncclReduceScatter C API.  The product is the C-ABI library
``vccl_amd/lib/libvccl.so`` (HIP for gfx950 + host C++); ``vccl_amd.nccl`` is
its ctypes binding.  See DESIGN.md and INTEGRATION.md.
"""
from . import nccl  # noqa: F401

__all__ = ["nccl"]
