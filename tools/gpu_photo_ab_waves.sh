set -o pipefail
mkdir -p gpurun_out/r03p
for so in w2 w3; do
 for R in 20 28; do
  USF_LIB=$(pwd)/unsamflow_amd/lib/ab/lib_$so.so USF_PHOTO_ROWS=$R timeout -k 10 200 python tools/photoab.py --out gpurun_out/r03p/ab_${so}_$R.json > gpurun_out/r03p/ab_${so}_$R.log 2>&1 || { tail gpurun_out/r03p/ab_${so}_$R.log; exit 1; }
  echo "== $so R=$R"; grep -v amdgpu gpurun_out/r03p/ab_${so}_$R.log | head -2
 done
done
