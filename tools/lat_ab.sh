#!/bin/bash
# Latency A/B of library builds: the 128-set call under a kernel trace per build.
#   LIBS="base: rdummy:lodestar_amd/_native/liblodestar_bls_rdummy.so ..."  (label:path; empty = default)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-lat_ab}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for ab in $LIBS; do
  label=${ab%%:*}; lib=${ab#*:}
  if [ -n "$lib" ]; then export LODESTAR_BLS_LIB=$R/$lib; else unset LODESTAR_BLS_LIB; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$label -o run --output-format csv -- python3 $R/tools/lat_probe.py --runs 10 --no-check > $O/$label.log 2>&1 || { tail -20 $O/$label.log; exit 1; }
  python3 -c "
import csv,glob,json
f=glob.glob('$O/$label/**/*kernel_stats.csv',recursive=True)[0]
d={r['Name'].split('(')[0]:round(float(r['AverageNs'])/1e3,1) for r in csv.DictReader(open(f)) if r['Name'].startswith(('k_pset','k_pre','k_indiv','k_fold'))}
print('$label', open('$O/$label.log').read().strip().splitlines()[-1][:60], d)"
done
