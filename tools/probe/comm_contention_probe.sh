# One-GPU A/B of the CU reservation for a concurrent comm kernel (cu_reserve.hip):
#   base   : the BERT-base phase-1 step alone
#   load   : + a stand-in comm kernel of R workgroups (48 KiB LDS each: no GEMM workgroup fits
#            beside one), dealt over the 8 XCDs like an RCCL kernel's channels, spinning for ~40 of
#            the ~52 ms step on its own stream; plans still assume every CU
#   (an earlier form confined the load to CU-mask bits 0..R-1 with hipExtStreamCreateWithCUMask:
#    the whole step ran 1.85x, with or without the reservation -- consistent with those CUs
#    sitting in one XCD, whose share of every GEMM then ran at half speed;
#    profiles/r3_comm_contention_masked.log)
#   load+R : the same load, plans sized for 256 - R CUs (--reserve-cus R)
# usage: bash tools/probe/comm_contention_probe.sh [R] > gpurun_out/comm_contention.log
set -o pipefail
R=${1:-16}
for rnd in 1 2; do
  for cfg in base load loadR; do
    case $cfg in
      base) extra="" ;;
      load) extra="--comm-load $R:40000:48" ;;
      loadR) extra="--comm-load $R:40000:48 --reserve-cus $R" ;;
    esac
    echo "== round $rnd $cfg (R=$R)"
    timeout -k 10 300 python -u bench.py --steps 12 --warmup 4 $extra 2>&1 | grep '^{"metric"' || exit 1
  done
done
