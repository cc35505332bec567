# DR routing passes: XCD-aware block order (default) vs plain (SRF_XCD_REMAP=0), C4 + C2,
# after the DR parity tests.   TAG=name bash scripts/gpu_xcd_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-xcd}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_route_dr_gpu.py tests/test_model_gpu.py -q --timeout 200 --timeout-method thread -k "not sdr and not c3 and not c5" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for x in 1 0; do
  SRF_XCD_REMAP=$x timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/b_x${x}_$rep.json 2> $OUT/b_x${x}_$rep.err || { tail -3 $OUT/b_x${x}_$rep.err; exit 1; }
  python -c "
import json; d=json.load(open('$OUT/b_x${x}_$rep.json')); e=d['extra']['timit_c2']
print('xcd=$x', 'C4', d['ms_per_step'], 'frac', d['roofline']['frac'], 'C2', e['ms_per_step'], e['roofline']['frac'])"
done
done
