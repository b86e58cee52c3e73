# round 6 session 4: the whole GPU suite + smoke on this tree, the first camera upload of
# the 81,920-face mesh, and the XCD-aware block order on it (time A/B + HBM traffic).
O=gpurun_out/s4
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step pytest_gpu 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread
step smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()"
RTX_SETUP_LOG=1 step setup_blob 180 python -u tools/setup_probe.py blob1080
for rep in 1 2; do
  for x in 0 1; do
    RTX_XCD_MAP=$x step ab_xcd${x}_r$rep 200 python -u bench.py --config blob1080 --steps 200 --warmup 20 --no-cpu-baseline
  done
done
RTX_XCD_MAP=1 TAG=s4/pmc_blob_xcd CFG=blob1080 PMC_GROUPS="FETCH_SIZE
WRITE_SIZE" step pmc_blob_xcd 300 bash tools/pmc_session.sh
echo done
