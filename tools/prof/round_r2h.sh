# r2h: rocprofv3 kernel trace + PMC passes of the r2e product (edge-policy lean rows), 1 M x 1500 B
set -e
timeout -k 10 900 bash tools/prof/profile.sh r2h mtu1500 > gpurun_out/r2h_profile.log 2>&1
echo done
