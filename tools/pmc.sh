#!/bin/bash
# Counter passes (one rocprofv3 --pmc run per pass; never combined with other traces).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PMC_NAME:-pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CMD=${PMC_CMD:-"$R/tools/conv_microbench.py 5"}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for pass in "${PMC_PASSES[@]:-}"; do :; done
for pass in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/pass$i -o run -- python3 $CMD > $OUT/pass$i.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "pass $i ($pass) rc=$rc"; tail -5 $OUT/pass$i.log; exit $rc; fi
done
echo done
