export ESGD_TIMEOUT_S=60
O=gpurun_out/r05ai
mkdir -p $O
bash tools/gpu_steps.sh $O \
  "400 python -u tools/long_stress.py --pipelined 2:64,4:mix,8:mix --rounds 8000 > $O/long_stress_pipelined.jsonl" \
  "300 python -u tools/long_stress.py --pipelined 3:mix --strict 1 --rounds 6400 > $O/long_stress_pipelined_strict.jsonl"
