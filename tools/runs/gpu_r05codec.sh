# codec A/B: tests under the default build, then encode/decode times of
# $VARIANTS builds (lib/variants, base = lib), then the multi-rank and RCCL
# tests under the default.
set -o pipefail
R="$GRAFT_REPO_ROOT"; O="$R/gpurun_out/codec"; mkdir -p "$O"; cd "$R"
V="$R/parallel-computing-mpi_amd/lib/variants"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_codec.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_codec.log" 2>&1 || { tail -30 "$O/pytest_codec.log"; exit 1; }
tail -1 "$O/pytest_codec.log"
for rep in 1 2; do
  for v in ${VARIANTS:-bpw1 bpw8 base}; do
    if [ $v = base ]; then unset MISORT_LIBRARY; else export MISORT_LIBRARY=$V/libmisort_$v.so; fi
    timeout -k 10 120 python3 -u tools/codec_probe.py > "$O/${v}_$rep.jsonl" || exit 1
    python3 -c "
import json
for l in open('$O/${v}_$rep.jsonl'):
    d=json.loads(l); print('$v', $rep, d['dtype'], d['keys'], 'enc %.3f dec %.3f ms ratio %.2f ok %s' % (d['encode_ms'], d['decode_ms'], d['ratio'], d['roundtrip_ok']))"
  done
done
unset MISORT_LIBRARY
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl_large.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/pytest_mr.log" 2>&1; rc=$?
tail -2 "$O/pytest_mr.log"; exit $rc
