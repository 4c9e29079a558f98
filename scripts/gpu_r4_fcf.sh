set -u
# (DQN_FCF was a temporary switch for this A/B; the launcher now picks by block count)
OUT=gpurun_out/r4fcf; mkdir -p $OUT
for rep in 1 2; do for x in 0 1 2; do
  DQN_FCF=$x timeout -k 10 300 python bench.py --variant rainbow --steps 2000 --warmup 200 > $OUT/rb_f${x}_$rep.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('$OUT/rb_f${x}_$rep.log').read().strip().splitlines()[-1]); print('rainbow fcf=$x rep=$rep', d['value'], d['ms_per_step'])"
done; done
