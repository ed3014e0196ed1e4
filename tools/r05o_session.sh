export ESGD_TIMEOUT_S=60
O=gpurun_out/r05o
mkdir -p $O/hang
export ESGD_HANG_DUMP_DIR=$O/hang ESGD_HANG_DUMP_S=60 ESGD_PROGRESS_FILE=$O/progress.txt
bash tools/gpu_steps.sh $O \
 "300 python -u tools/long_stress.py --pipelined 2:64,4:mix --rounds 1000 >> $O/soak.jsonl" \
 "400 python -u tools/long_stress.py --pipelined 8:mix --rounds 800 >> $O/soak.jsonl" \
 "300 python -u tools/long_stress.py --pipelined 3:mix --rounds 800 --strict 1 >> $O/soak.jsonl" \
 "300 python -u tools/long_stress.py --pipelined 8:mix --rounds 400 --fail-exports 0,0,0,0,1,1,1,1 --kinds majority >> $O/soak.jsonl"
