set -o pipefail
OUT=gpurun_out/lm1; mkdir -p $OUT
for r in 1 2; do for wl in config2 config5 config3; do for lm in 64 96 128 192; do
  HPK_LIB=loona_amd/libhpk_diag.so HPK_LONG_MIN=$lm timeout -k 10 180 python scripts/dec_time.py $wl 20 > $OUT/one.json 2>>$OUT/err.log || { echo "failed $wl $lm"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$OUT/one.json').read().strip().splitlines()[-1]); d['long_min_env']=$lm; print(json.dumps(d))" >> $OUT/lm.jsonl
done; done; done
python3 -c "
import json
for l in open('$OUT/lm.jsonl'):
    d=json.loads(l); print(d['workload'], d['long_min_env'], d['decode_us'], d['checked'])"
