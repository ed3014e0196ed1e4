# round 3 session D: esgd with the arena bypassed, both lifetimes; the -m gpu suite; N=1 bench
O=gpurun_out/r03d; mkdir -p $O
timeout -k 10 300 python -u tools/ipc_bisect.py --only none > $O/ipc_bisect_esgd.txt 2>&1
rc=$?; echo "bisect rc=$rc" >> $O/ipc_bisect_esgd.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/gpu_session.sh r03d n1
