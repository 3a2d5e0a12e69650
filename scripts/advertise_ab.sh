# A/B of the claim path's device-plugin advertisement on real hardware: strict (mark advertised
# after gRPC reports the ListAndWatch write complete; GPUPOOL_ADVERTISE_ON_WRITE=1) vs on submit
# (the default). Headline bench, 2 interleaved runs each, claim span breakdown kept.
set -o pipefail
O=gpurun_out/${1:-advab}
mkdir -p $O
for r in 1 2; do
  for mode in write submit; do
    if [ $mode = write ]; then export GPUPOOL_ADVERTISE_ON_WRITE=1; else unset GPUPOOL_ADVERTISE_ON_WRITE; fi
    timeout -k 10 300 python -u bench.py --steps 15 --warmup 2 --scale-down-steps 0 --pool-steps 0 \
      --health-steps 0 --fault-steps 0 --azure-steps 0 > $O/bench_${mode}_$r.json 2> $O/bench_${mode}_$r.err || exit $?
  done
done
