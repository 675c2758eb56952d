set -u
mkdir -p gpurun_out
A="timeout -k 10 240 python -u tools/ab_tune.py"
$A --graph reddit --reduce max --weighted 0 --configs "base;v4:flat_vec_arg=4;v1:flat_vec_arg=1" > gpurun_out/ab_vec_c4.log 2>&1 || exit $?
$A --graph reddit --reduce sum --configs "base;v2:flat_vec1_min_bytes=1099511627776;v4:flat_vec1_min_bytes=1099511627776,flat_vec=4" >> gpurun_out/ab_vec_c4.log 2>&1 || exit $?
$A --graph rmat21 --reduce max --weighted 0 --configs "base;v4:flat_vec_arg=4" >> gpurun_out/ab_vec_c4.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/ab_vec_c4.log
