set -o pipefail
# Round 3, pass d: cost of the completion word in the pack/unpack kernels; fixed grids.
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 180 ./tools/pack_variants > $O/pack_variants.txt 2> $O/pack_variants.err || { tail -5 $O/pack_variants.err; exit 1; }
grep -E "done|pair|ref:" $O/pack_variants.txt
