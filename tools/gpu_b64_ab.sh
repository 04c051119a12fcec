set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; mkdir -p gpurun_out
PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/r64b8/libplvi_frontend.so timeout -k 10 300 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread -k "lines or frame" > gpurun_out/r64_tests.log 2>&1; rc=$?; echo "tests: $(tail -1 gpurun_out/r64_tests.log)"; [ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do for v in base r64b4 r64b8 r64b16; do
  if [ $v = base ]; then unset PLVI_LIB; else export PLVI_LIB=$R/pl-vi-orbslam3_amd/variants/$v/libplvi_frontend.so; fi
  out=$(timeout -k 10 120 python -u tools/b64_probe.py 64 60 2>/dev/null | tail -1); rc=$?; echo "$v $out"; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
