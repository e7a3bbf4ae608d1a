#!/usr/bin/env bash
# end-of-round evidence: full GPU suite (no -x), smoke(), headline + transformer benches
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r6final
rm -rf $out && mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 150 --timeout-method thread > $out/tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $out/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || exit $?
for m in resnet50 bert_large gpt2_medium; do
  timeout -k 10 300 python -u bench.py --model $m --steps 30 --warmup 10 --json-out $out/$m.json > $out/$m.log 2>&1 || exit $?
done
timeout -k 10 300 python -u bench.py --steps 30 --warmup 10 --json-out $out/resnet50_2.json > $out/resnet50_2.log 2>&1
exit $rc
