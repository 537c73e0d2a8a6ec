set -e
mkdir -p gpurun_out
for lib in liblneto_amd liblneto_amd_nt liblneto_amd_sc1 liblneto_amd_sc0sc1 liblneto_amd_ntsc1; do
  LNETO_AMD_LIB=$PWD/lneto_amd/$lib.so timeout -k 10 120 python tools/prof/variants.py mtu1500 0,10,0,1 
done
