#!/usr/bin/env python3
"""Generate tests/golden/functable.json from the REFERENCE's own generator.

Runs /root/reference/src/device/generate.py (the reference's only Python file)
as a subprocess into a scratch directory and records, for every
AllReduce / ReduceScatter row, the primary device-function id it maps to
(ncclDevFuncRowToId in the generated host_table.cc).  Rows sharing an id run
the same kernel: this pins the signed->unsigned equivalence
(generate.py:129-137) and the unsupported combinations (id -1, e.g.
SumPostDiv on floats, generate.py:99-125) that our dispatch must reproduce.

Only run in the build container (the reference is absent on the GPU box);
the JSON it writes is the committed fixture.
"""
import json
import os
import re
import subprocess
import sys
import tempfile

REF_GEN = "/root/reference/src/device/generate.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "functable.json")


def main():
    with tempfile.TemporaryDirectory() as d:
        gensrc = os.path.join(d, "gensrc")
        subprocess.check_call([sys.executable, REF_GEN, gensrc, ""],
                              cwd=os.path.dirname(REF_GEN))
        text = open(os.path.join(gensrc, "host_table.cc")).read()
    body = text.split("ncclDevFuncRowToId[] = {", 1)[1].split("};", 1)[0]
    rows = []
    pat = re.compile(r"/\*\s*(\d+)\*/\s*(-?\d+),\s*(?://\s*(.*))?")
    for line in body.strip().splitlines():
        m = pat.search(line)
        if not m:
            continue
        row, fid, name = int(m.group(1)), int(m.group(2)), (m.group(3) or "").strip()
        rows.append({"row": row, "id": fid, "name": name})
    # Unnamed rows (-1) still have a deterministic (coll, redop, ty, algo, proto)
    # from enumerate_func_rows(); recover it by re-enumerating the same lists.
    colls_red = ("AllReduce", "Reduce", "ReduceScatter")
    all_redops = ["Sum", "Prod", "MinMax", "PreMulSum", "SumPostDiv"]
    all_tys = ["i8", "u8", "i32", "u32", "i64", "u64", "f16", "f32", "f64", "bf16",
               "f8e4m3", "f8e5m2"]
    all_protos = ["LL", "LL128", "SIMPLE"]
    algos_of = {"AllGather": ["RING", "COLLNET_DIRECT", "NVLS", "PAT"],
                "Broadcast": ["RING"],
                "AllReduce": ["TREE", "RING", "COLLNET_DIRECT", "COLLNET_CHAIN", "NVLS",
                              "NVLS_TREE"],
                "Reduce": ["RING"],
                "ReduceScatter": ["RING", "COLLNET_DIRECT", "NVLS", "PAT"]}
    enum = [("SendRecv", None, None, None, None)]
    for c in ("AllGather", "Broadcast"):
        for a in algos_of[c]:
            for p in all_protos:
                enum.append((c, None, None, a, p))
    for c in colls_red:
        for r in all_redops:
            for t in all_tys:
                for a in algos_of[c]:
                    for p in all_protos:
                        enum.append((c, r, t, a, p))
    assert len(enum) == len(rows), (len(enum), len(rows))
    keep = []
    for (c, r, t, a, p), row in zip(enum, rows):
        if row["name"]:
            assert row["name"] == " ".join(x for x in (c, r, t, a, p) if x), row
        if c in ("AllReduce", "ReduceScatter", "AllGather") and a in ("RING", "TREE"):
            keep.append({"row": row["row"], "id": row["id"], "coll": c, "redop": r,
                         "type": t, "algo": a, "proto": p})
    json.dump({"source": "reference src/device/generate.py (run unmodified)",
               "rows": keep}, open(OUT, "w"), indent=0)
    print(f"wrote {OUT}: {len(keep)} rows")


if __name__ == "__main__":
    main()
