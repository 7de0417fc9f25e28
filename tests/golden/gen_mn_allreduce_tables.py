"""Writes tests/golden/mn_allreduce_tables.json: the multi-node allreduce tuning tables MVAPICH2
falls back to (allreduce_tuning.c default branch: tuning/allreduce/
nemesis_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h), as data: per numproc entry the
is_two_level flags, the inter-leader and the intra-node function per message-size index (the
first size_inter_table / size_intra_table = 18 entries, 1 B ... 128 KiB).  Letters: s pt2pt_rs,
d pt2pt_rd, m the multicast helper (falls back to pt2pt_rd here), h reduce_shmem, p reduce_p2p.

Run in the container that holds the reference (python tests/golden/gen_mn_allreduce_tables.py);
the tests read only the JSON."""
import json
import os
import re
import sys

REF = os.environ.get("MV2_REFERENCE", "/root/reference")
DIR = os.path.join(REF, "src", "mpi", "coll", "tuning", "allreduce")
FN = {"pt2pt_rs_MV2": "s", "pt2pt_rd_MV2": "d", "mcst_reduce_two_level_helper_MV2": "m",
      "reduce_shmem_MV2": "h", "reduce_p2p_MV2": "p"}
ENTRY = re.compile(r"\{\s*(\d+),\s*(\d+),\s*\{([\d,\s]+)\},\s*(\d+),\s*\{(.*?)\},\s*(\d+),\s*\{(.*?)\}\s*\}", re.S)


def read(conf):
    text = open(os.path.join(DIR, f"nemesis_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{conf}.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text.replace("\\", ""), flags=re.S)
    out = []
    for m in ENTRY.finditer(text):
        numproc, _mcast, bits, ninter, inter, nintra, intra = m.groups()
        fns = lambda body: "".join(FN[f.replace("MPIR_Allreduce_", "")] for f in re.findall(r"&(\w+)", body))
        out.append({"numproc": int(numproc), "two_level": "".join(bits.split()).replace(",", "")[:int(ninter)],
                    "inter": fns(inter)[:int(ninter)], "intra": fns(intra)[:int(nintra)]})
    return out


def main():
    tables = {conf: read(conf) for conf in ("1ppn", "2ppn", "16ppn")}
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mn_allreduce_tables.json")
    with open(dst, "w") as f:
        json.dump(tables, f, indent=1)
    print(dst, {k: [e["numproc"] for e in v] for k, v in tables.items()}, file=sys.stderr)


if __name__ == "__main__":
    main()
