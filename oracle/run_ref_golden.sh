#!/bin/bash
# Run on an MI355X box (gpurun): the reference kernels on the golden inputs,
# twice (runs A and B must agree bit for bit), plus one 1080p pair whose
# outputs and kernel times are kept under gpurun_out/ (too big to commit).
set -euo pipefail
cd "$(dirname "$0")/.."
D=gpurun_out/golden_in
H=oracle/_ref/ref_harness_hip
python tests/golden/make_golden.py prepare $D
for t in A B; do
  awk -v t=$t '{$7=$7"_"t; print}' $D/jobs.txt > $D/jobs_$t.txt
  timeout -k 10 300 $H oracle/_ref/affine_2cp.co oracle/_ref/affine_3cp.co $D/jobs_$t.txt > gpurun_out/ref_run_$t.log 2>&1
done
python tests/golden/make_golden.py prepare1080 gpurun_out/ref1080
timeout -k 10 300 $H oracle/_ref/affine_2cp.co oracle/_ref/affine_3cp.co gpurun_out/ref1080/jobs.txt > gpurun_out/ref_run_1080.log 2>&1
cat gpurun_out/ref_run_A.log gpurun_out/ref_run_1080.log
echo done
