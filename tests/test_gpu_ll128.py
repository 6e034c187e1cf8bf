"""LL128-style line tearing probe on the GPU (tools/line_probe.hip).

VCCL's LL128 trusts a 128-byte line's 15 data words once its flag word shows
the step (src/device/prims_ll128.h:176-324).  The probe writes lines with sc0
sc1 16-byte stores from one XCD and polls them from another, counting lines
whose flag is visible before their data.  Both line sizes run: 64 B (the
LL128 ring's line, one 64-byte write request per flag) must never tear; 128 B
(VCCL's NVLink line, two write requests) is measured only — it tore in
profiles/r04l (a parity run) and r04m (8 of 163,840,000 probe lines).
"""
import ctypes
import json
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

if not torch.cuda.is_available():
    pytest.skip("needs a GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("line_bytes", [128, 64])
def test_line_tearing_probe(line_bytes):
    L = ctypes.CDLL(os.path.join(ROOT, "vccl_amd", "lib", "libvccl_probe.so"))
    L.vcclProbeLineTearing.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_double, ctypes.POINTER(ctypes.c_ulonglong)]
    pairs, lines, iters = 64, 128, 20000
    counts = (ctypes.c_ulonglong * 4)()
    rc = L.vcclProbeLineTearing(pairs, lines, iters, line_bytes, 20.0, counts)
    assert rc == 0, rc
    checked, flag_first, data_ahead, timeouts = list(counts)
    rec = {"line_bytes": line_bytes, "pairs": pairs, "lines_per_pair": lines, "iters": iters,
           "lines_checked": checked, "flag_before_data": flag_first,
           "data_ahead_of_flag": data_ahead, "timeouts": timeouts}
    print(json.dumps(rec))
    out = os.path.join(ROOT, "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, f"line_probe_{line_bytes}.json"), "w") as f:
        json.dump(rec, f)
    assert timeouts == 0
    assert checked == pairs * lines * iters
    assert data_ahead == 0  # the writer waits for the reader's acknowledgement
    if line_bytes == 64:  # the shipped LL128 line
        assert flag_first == 0, rec
