# Round 3 session o: the relaxed counters / gate of k_round_small -- the GPU suite, the
# writer-then-post visibility worker with ranks sharing the GPU (one- and five-launch
# rounds, every flag kind), then the N = 2 / 4 rehearsal lines (small-round latency, C4
# 161-bucket chain).  The first failure ends the session.
set -e
T=${1:-r03o}
O=gpurun_out/$T; mkdir -p $O
bash tools/gpu_session.sh $T
timeout -k 10 240 python -u -c "
import sys; sys.path.insert(0, 'tests'); import mp_workers as m
for kw in (dict(world=2, flag_mode=0, count=65539), dict(world=2, flag_mode=1, count=65539),
           dict(world=3, flag_mode=2, count=65539), dict(world=8, flag_mode=0, count=65539),
           dict(world=4, flag_mode=0, small_bytes=0)):
    w = kw.pop('world'); print(w, kw, m.run('gpu_visibility', w, **kw), flush=True)
" > $O/visibility_shared_gpu.txt 2>&1
bash tools/bench_round.sh $T n2 n4
