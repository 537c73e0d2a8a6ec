# r2w: rocprofv3 kernel trace + PMC passes of the r2 product on the jumbo and Zipf workloads
set -e
timeout -k 10 900 bash tools/prof/profile.sh r2w jumbo9000 > gpurun_out/r2w_profile_jumbo.log 2>&1
timeout -k 10 900 bash tools/prof/profile.sh r2w zipf64_1500 > gpurun_out/r2w_profile_zipf.log 2>&1
echo done
