# one-off steps of this round (run through gpurun from the repo root)
set -o pipefail
mkdir -p gpurun_out
T=${T:-r04zf}
SMX_LIB=scann_amd/lib/libscann_mi355x.so timeout -k 10 300 python tools/tune.py 0,1,0,20 0,2,0,20 0,3,0,20 0,4,0,20 0,5,0,20 0,6,0,20 0,8,0,20 0,4,0,20 > gpurun_out/$T.tune.log 2>&1
