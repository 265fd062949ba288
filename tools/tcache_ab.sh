set -e
mkdir -p gpurun_out/tcache_ab
for rep in 1 2; do
for tc in 7 64 256 1024; do
  GLIBC_TUNABLES="glibc.malloc.tcache_count=$tc:glibc.malloc.tcache_max=16384" timeout -k 10 300 python -u bench.py --steps 300 --warmup 5 --report-cpu --json-out gpurun_out/tcache_ab/tc${tc}_r${rep}.json > gpurun_out/tcache_ab/tc${tc}_r${rep}.log 2>&1
  echo "tc=$tc rep=$rep done"
done
done
