"""Writes tests/golden/mn_reduce_tables.json: the multi-node reduce tuning tables MVAPICH2 falls
back to for an unlisted architecture (reduce_tuning.c:1563-1649, the "Stampede" branch:
tuning/reduce/gen2{_cma}_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{1,2,16}ppn.h, of which the first 5 / 6 / 6
numproc entries are used), as data: per numproc entry inter_k_degree, intra_k_degree, the
is_two_level_reduce flags, and the inter-leader and intra-node function per message-size index (the
first size_inter_table / size_intra_table entries) with each list's smallest message size.  Letters:
b MPIR_Reduce_binomial_MV2, k MPIR_Reduce_inter_knomial_wrapper_MV2, i MPIR_Reduce_intra_knomial_
wrapper_MV2, r MPIR_Reduce_redscat_gather_MV2, h MPIR_Reduce_shmem_MV2.

Run in the container that holds the reference (python tests/golden/gen_mn_reduce_tables.py); the
tests read only the JSON."""
import json
import os
import re
import sys

REF = os.environ.get("MV2_REFERENCE", "/root/reference")
DIR = os.path.join(REF, "src", "mpi", "coll", "tuning", "reduce")
FN = {"binomial": "b", "inter_knomial_wrapper": "k", "intra_knomial_wrapper": "i", "redscat_gather": "r",
      "shmem": "h"}
USED = {"1ppn": 5, "2ppn": 6, "16ppn": 6}  # mv2_size_reduce_indexed_tuning_table[] (reduce_tuning.c:1582-1626)
ENTRY = re.compile(r"\{\s*(\d+),\s*(\d+),\s*(\d+),\s*\{([\d,\s]+)\},\s*(\d+),\s*\{(.*?)\},\s*(\d+),\s*\{(.*?)\}\s*\}", re.S)
ELEM = re.compile(r"\{\s*(\d+),\s*&MPIR_Reduce_(\w+)_MV2\s*\}")


def read(name):
    text = open(os.path.join(DIR, name)).read()
    text = re.sub(r"/\*.*?\*/", "", text.replace("\\", ""), flags=re.S)
    out = []
    for m in ENTRY.finditer(text):
        numproc, kinter, kintra, bits, ninter, inter, nintra, intra = m.groups()
        ie, ne = ELEM.findall(inter), ELEM.findall(intra)
        out.append({"numproc": int(numproc), "inter_k": int(kinter), "intra_k": int(kintra),
                    "two_level": "".join(bits.split()).replace(",", "")[:int(ninter)],
                    "inter_min": int(ie[0][0]), "inter": "".join(FN[f] for _, f in ie[:int(ninter)]),
                    "intra_min": int(ne[0][0]), "intra": "".join(FN[f] for _, f in ne[:int(nintra)])})
    return out


def main():
    tables = {}
    for cma in ("cma", "nocma"):
        for conf, used in USED.items():
            name = f"gen2{'_cma' if cma == 'cma' else ''}_INTEL_XEON_E5_2680_16_MLX_CX_FDR_{conf}.h"
            tables[f"{cma}_{conf}"] = read(name)[:used]
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "mn_reduce_tables.json")
    with open(dst, "w") as f:
        json.dump(tables, f, indent=1)
    print(dst, {k: [e["numproc"] for e in v] for k, v in tables.items()}, file=sys.stderr)


if __name__ == "__main__":
    main()
