# Per-dataset loglike_batch profiles at W=1024 (tools/cmbl_profile.py)
set -u
mkdir -p gpurun_out
rm -f gpurun_out/ds_prof.log
for c in lensing spt sptteee sptbb bk15 bk; do
  timeout -k 10 120 python -u tools/cmbl_profile.py $c 1024 30 >> gpurun_out/ds_prof.log 2>&1 || exit $?
done
grep -v amdgpu.ids gpurun_out/ds_prof.log
