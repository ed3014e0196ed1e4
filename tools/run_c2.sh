set -e
O=gpurun_out/c3; mkdir -p $O
gcc -O2 -std=c11 -Iinclude tests/c/ff_known_answers.c -o $O/ffka eager-sgd_amd/esgd/libesgd.so -Wl,-rpath,$PWD/eager-sgd_amd/esgd
J=dbg$$
for r in 0 1; do RANK=$r WORLD_SIZE=2 LOCAL_RANK=0 ESGD_JOB_ID=$J ESGD_TIMEOUT_S=60 ESGD_DEBUG=1 timeout -k 5 120 $O/ffka 10007 4 > $O/out$r.txt 2>&1 & done
wait
