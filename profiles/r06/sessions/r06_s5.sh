# round 6 session 5: primary-ray face lists through LDS (option bin_lds) -- exactness on the
# mesh tests and an A/B on the 81,920-face mesh and TorusMesh; the first camera upload of
# the 81,920-face mesh with the sorts warmed at scene creation.
O=gpurun_out/s5
mkdir -p $O
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  timeout -k 10 $to "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?
  echo "$name rc=$rc" >> $O/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc $rc)"; exit $rc; fi
}
RTX_BIN_LDS=1 step pytest_binlds 500 python -u -m pytest -v --timeout 120 --timeout-method thread "tests/test_gpu_parity.py::test_device_face_bins_equal_host" "tests/test_gpu_parity.py::test_heavy_tiles_equal_walk" "tests/test_gpu_parity.py::test_large_mesh_bvh_matches_oracle" "tests/test_gpu_parity.py::test_primary_bins_equal_walk" "tests/test_gpu_parity.py::test_config_size_1080p_matches_oracle" "tests/test_gpu_parity.py::test_render_matches_oracle" "tests/test_gpu_parity.py::test_counters_match_oracle_tallies"
RTX_SETUP_LOG=1 step setup_blob 180 python -u tools/setup_probe.py blob1080
for rep in 1 2; do
  for b in 0 1; do
    RTX_BIN_LDS=$b step ab_blob_l${b}_r$rep 200 python -u bench.py --config blob1080 --steps 200 --warmup 20 --no-cpu-baseline
    RTX_BIN_LDS=$b step ab_tm_l${b}_r$rep 200 python -u bench.py --config tm1080 --steps 500 --warmup 20 --no-cpu-baseline
  done
done
echo done
