set -o pipefail
run() { tag=$1; shift; env "$@" timeout -k 10 240 python bench.py --no-cpu-baseline --no-pmc --steps 8 --warmup 2 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err; }
run def H2G_X=0 && \
run main50 H2G_CU_MASK_MAIN=55555555,55555555,55555555,55555555,55555555,55555555,55555555,55555555 && \
run main25 H2G_CU_MASK_MAIN=11111111,11111111,11111111,11111111,11111111,11111111,11111111,11111111 H2G_CU_MASK_MSM=eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee && \
run main75 H2G_CU_MASK_MAIN=77777777,77777777,77777777,77777777,77777777,77777777,77777777,77777777 && \
run def2 H2G_X=0
