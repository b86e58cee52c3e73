# round 6 session 3: multi-frame graphs, LDS-staged chunk pass (A/B of chunk_mode on the
# 81,920-face mesh), first-camera breakdown of the device face bins, blob PMC.
# A step that fails its checks (rc 1) lets the next one run; anything else ends the script.
O=gpurun_out/s3
mkdir -p $O
T="python -u -m pytest -v --timeout 120 --timeout-method thread"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step pytest 400 $T "tests/test_gpu_frame_loop.py::test_frame_graph_replays_render_and_gather" "tests/test_gpu_parity.py::test_device_face_bins_equal_host" "tests/test_gpu_parity.py::test_heavy_tiles_equal_walk" "tests/test_gpu_parity.py::test_large_mesh_bvh_matches_oracle"
for rep in 1 2; do
  for m in 0 1 2 3; do
    RTX_CHUNK_MODE=$m step ab_chunk_m${m}_r$rep 200 python -u bench.py --config blob1080 --steps 200 --warmup 20 --no-cpu-baseline
  done
done
RTX_SETUP_LOG=1 step setup_blob 180 python -u tools/setup_probe.py blob1080
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 step bench_pipeline 300 python -u bench.py --pipeline --steps 2000 --warmup 20 --no-cpu-baseline
TAG=s3/pmc_blob CFG=blob1080 step pmc_blob 600 bash tools/pmc_session.sh
echo done
