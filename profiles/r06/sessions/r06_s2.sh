# round 6 session 2: the new GPU tests, the frame-graph probe, cold start, bench lines.
# A step that fails its checks (rc 1) lets the next one run; anything else ends the script.
mkdir -p gpurun_out/s2
T="python -u -m pytest -v --timeout 120 --timeout-method thread"
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > gpurun_out/s2/$name.out 2> gpurun_out/s2/$name.err
  local rc=$?
  echo "$name rc=$rc" >> gpurun_out/s2/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
step pytest_new 500 $T tests/test_gpu_frame_loop.py tests/test_gpu_jit_cache.py "tests/test_gpu_parity.py::test_edits_between_renders_match_oracle" "tests/test_gpu_parity.py::test_camera_changes_rerender" "tests/test_gpu_parity.py::test_device_face_bins_equal_host" "tests/test_gpu_parity.py::test_codegen_options_render_the_default_bytes" "tests/test_gpu_parity.py::test_heavy_tiles_equal_walk"
step graph 180 python -u tools/graph_gather_probe.py tsp1080 2000
step cold_tsp 120 python -u tools/coldstart_probe.py tsp1080
RTX_SETUP_LOG=1 step setup_blob 180 python -u tools/setup_probe.py blob1080
RTX_SETUP_LOG=1 RTX_DEV_BINS=0 step setup_blob_host 180 python -u tools/setup_probe.py blob1080
step bench 300 python -u bench.py --steps 200 --warmup 10
step bench_blob 300 python -u bench.py --config blob1080 --steps 100 --warmup 10 --no-cpu-baseline
MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 WORLD_SIZE=1 RANK=0 LOCAL_RANK=0 step bench_pipeline 300 python -u bench.py --pipeline --steps 2000 --warmup 20 --no-cpu-baseline
echo done
