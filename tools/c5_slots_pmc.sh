set -o pipefail
O=gpurun_out/r05c5pmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for V in packed align; do
  A=""; [ $V = align ] && A="--align"
  for P in FETCH_SIZE WRITE_SIZE "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    N=$(echo $P | tr ' ' '_')
    timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $O/${V}_$N -o run -- python3 tools/c5_share.py --steps 5 $A > $O/${V}_$N.log 2>&1 || { echo "fail $V $N"; tail -5 $O/${V}_$N.log; exit 1; }
  done
done
echo done
