set -u
mkdir -p gpurun_out
for v in gu4 gu6 gu12; do
  echo "== $v"
  MI355_MP_LIB=tools/variants/lib_$v.so timeout -k 10 200 python -u tools/ab_gat_tile.py --vecs 0,4 --rounds 3 2>&1 | grep -v amdgpu.ids || exit $?
done
