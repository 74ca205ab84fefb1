set -u
out=$GRAFT_REPO_ROOT/gpurun_out/s03
mkdir -p $out
cd /tmp; export TMPDIR=/tmp
timeout -k 5 60 rocprofv3 -L > $out/avail.txt 2>&1 || true
for v in 6 12; do
  for pass in "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_DRAM_sum" "FETCH_SIZE" "WRITE_SIZE"; do
    tag=$(echo "$pass" | tr ' ' '_')
    ACSIM_BIN_POL=$v timeout -s KILL 90 rocprofv3 --pmc $pass --output-format csv -d $out/pol$v/$tag -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --legs= --steps 20 --warmup 2 > $out/pol${v}_$tag.log 2>&1
    echo "pol $v pass $pass rc=$?"
  done
done
