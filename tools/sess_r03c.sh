set -e
O=gpurun_out/r03c; mkdir -p $O
timeout -k 10 300 python -u tools/ipc_bisect.py --only late-close,late-close+engine,late-close-3 --no-esgd > $O/ipc_bisect_late.txt 2>&1
timeout -k 10 200 python -u -c "
import sys; sys.path.insert(0, 'tests'); import mp_workers as m
for kw in (dict(world=2, flag_mode=0), dict(world=2, flag_mode=1, count=65539), dict(world=3, flag_mode=2, small_bytes=0), dict(world=4, flag_mode=0, small_bytes=0)):
    w = kw.pop('world'); print(w, kw, m.run('gpu_visibility', w, **kw), flush=True)
" > $O/visibility_shared_gpu.txt 2>&1
