"""Writes tests/golden/red_scat_table.json: MPIR_Reduce_scatter_MV2's default tuning table (the
branch red_scat_tuning.c takes for an unlisted architecture: `mv2_size_red_scat_tuning_table = 7`),
as data: per entry numproc and its [min, max, function] rows (max -1 = unbounded).  Run in the
container that holds the reference; the tests read only the JSON."""
import json
import os
import re

REF = os.environ.get("MV2_REFERENCE", "/root/reference")
SRC = os.path.join(REF, "src", "mpi", "coll", "red_scat_tuning.c")
FN = {"MPIR_Reduce_Scatter_Basic_MV2": "rs_basic", "MPIR_Reduce_scatter_Rec_Halving_MV2": "rs_rec_halving",
      "MPIR_Reduce_scatter_Pair_Wise_MV2": "rs_pairwise", "MPIR_Reduce_scatter_ring_2lvl": "rs_ring",
      "MPIR_Reduce_scatter_ring": "rs_ring"}


def main():
    text = open(SRC).read()
    start = text.index("mv2_size_red_scat_tuning_table = 7;")
    body = text[text.index("thresholds_table[] = {", start):]
    body = body[:body.index("};")]
    # {numproc, size_inter_table, { rows }}: size_inter_table bounds the selection loop
    # (red_scat_osu.c:1877-1884) even where the entry lists more rows (numproc 128 / 256 / 512 list
    # three and declare two), so both are kept
    entries = []
    heads = list(re.finditer(r"\{\s*(\d+),\s*(\d+),\s*\{", body))
    for i, h in enumerate(heads):
        seg = body[h.end():heads[i + 1].start() if i + 1 < len(heads) else len(body)]
        rows = [[int(a), int(b), FN[f]] for a, b, f in re.findall(r"\{\s*(-?\d+),\s*(-?\d+),\s*&(\w+)\s*\}", seg)]
        entries.append({"numproc": int(h.group(1)), "size": int(h.group(2)), "rows": rows})
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "red_scat_table.json")
    with open(dst, "w") as f:
        json.dump({"ring_threshold": 131072, "entries": entries}, f, indent=1)
    print(dst, [e["numproc"] for e in entries])


if __name__ == "__main__":
    main()
