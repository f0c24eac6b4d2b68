set -o pipefail
mkdir -p gpurun_out/exp1
for v in default notail notail_nodirty; do
  if [ $v = default ]; then L=panman_amd/libpanman_amd.so; else L=build_var/$v/libpanman_amd.so; fi
  PANMAN_AMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu --with none --steps 10 --warmup 3 > gpurun_out/exp1/$v.json 2> gpurun_out/exp1/$v.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/exp1/$v.json'));r=d['roofline'];print('$v', round(d['ms_per_step'],3), r['kernel'], r['kernel_ms_per_step'], r['other_kernels_ms_per_step'])"
done
