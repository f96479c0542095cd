#!/bin/bash
# p50 of one call alone at several sizes, per-set path (BLS_SIGAGG=0) vs aggregated (=1)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-lat_sizes}
mkdir -p $O
for n in ${SIZES:-512 1024 2048 4096}; do
  for sa in 0 1; do
    BLS_SIGAGG=$sa timeout -k 10 120 python3 $R/tools/lat_probe.py --sets $n --batchable --runs 7 > $O/n${n}_sigagg${sa}.json 2> $O/n${n}_sigagg${sa}.err || { tail -5 $O/n${n}_sigagg${sa}.err; exit 1; }
    echo "n=$n sigagg=$sa $(cat $O/n${n}_sigagg${sa}.json)"
  done
done
