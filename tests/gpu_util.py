"""Device-memory plumbing for the GPU tests (torch is only the allocator)."""
import numpy as np
import torch


def to_dev(a: np.ndarray, pad: int = 0, offset: int = 0) -> tuple[torch.Tensor, int]:
    """Copy `a` to a fresh device byte buffer; returns (tensor, data pointer).

    `offset` shifts the data start by that many bytes (misalignment tests)."""
    raw = np.ascontiguousarray(a).view(np.uint8).reshape(-1)
    t = torch.zeros(raw.size + pad + offset + 256, dtype=torch.uint8, device="cuda")
    t[offset:offset + raw.size].copy_(torch.from_numpy(raw.copy()))
    return t, t.data_ptr() + offset


def empty_dev(nbytes: int, offset: int = 0, fill: int = 0xA5) -> tuple[torch.Tensor, int]:
    t = torch.full((nbytes + offset + 256,), fill, dtype=torch.uint8, device="cuda")
    return t, t.data_ptr() + offset


def from_dev(t: torch.Tensor, dtype, n: int, offset: int = 0) -> np.ndarray:
    nbytes = n * np.dtype(dtype).itemsize
    return t[offset:offset + nbytes].cpu().numpy().view(dtype).copy()


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream
