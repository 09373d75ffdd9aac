timeout -k 10 60 ./tools/csrc/mfma_f64_layout > gpurun_out/mfma_f64_layout.txt 2>&1
bash tools/gpu_r4b.sh r4b; rc=$?; if [ $rc -eq 0 ]; then bash tools/gpu_als_diag.sh r4als; rc=$?; fi; exit $rc
