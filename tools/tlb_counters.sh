# Why 8 x 1 GiB runs below 8 x 256 MiB: translation (UTCL1 / UTCL2)
# and traffic counters of the production reduction at both shapes, one rocprofv3 --pmc
# pass per counter group (gfx950 slots: 4 TCP, 2 GRBM, 4 TCC -- FETCH_SIZE and WRITE_SIZE
# in passes of their own), plus a kernel-trace pass for per-window durations.  The
# program is bench.py's PMC child: PMC_CALLS (5) calls of 8 inputs -> 1 output, 64 MiB
# windows.  Summarised by tools/tlb_summary.py.
#   bash tools/tlb_counters.sh <tag>
O=gpurun_out/${1:-tlb}; mkdir -p $O; R=$PWD
cd /tmp && export TMPDIR=/tmp
P1="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_PERMISSION_MISS_sum GRBM_UTCL2_BUSY GRBM_GUI_ACTIVE"
P2="TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum"
P3="TCP_UTCL1_STALL_LFIFO_NO_RES_sum TCP_UTCL1_LFIFO_FULL_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_CLIENT_UTCL1_INFLIGHT_sum"
# memory side (passes 7, 8): read / write requests and their in-flight sums (average
# latency = LEVEL / requests), DRAM-credit stalls
P7="TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_WRREQ_sum"
P8="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_STALL_sum TCC_EA0_RDREQ_DRAM_sum"
# TLB_PASSES="7 8" runs only those passes (the numbering of the full list is kept)
for mib in 256 1024; do
  i=0
  for pass in "$P1" "$P2" "$P3" FETCH_SIZE WRITE_SIZE trace "$P7" "$P8"; do
    i=$((i + 1))
    if [ -n "$TLB_PASSES" ] && ! echo " $TLB_PASSES " | grep -q " $i "; then continue; fi
    d=$R/$O/${mib}MiB_p$i
    if [ "$pass" = trace ]; then
      timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $d -o kt -- \
          python3 $R/bench.py --pmc-child 1 --bucket-mib $mib > $d.log 2>&1
    else
      timeout -s KILL 150 rocprofv3 --pmc $pass --output-format csv -d $d -o pmc -- \
          python3 $R/bench.py --pmc-child 1 --bucket-mib $mib > $d.log 2>&1
    fi
    rc=$?
    echo "$mib MiB pass $i ($pass): rc=$rc" >> $R/$O/passes.txt
    # a counter this chip lacks fails its pass (rc 1); a kill, fault or abort ends the session
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  done
done
cd $R && python3 tools/tlb_summary.py $O > $O/tlb_summary.json
