set -u
timeout -k 10 300 tools/fdiv_exhaust 64 > gpurun_out/fdiv_exhaust2.txt 2>&1; echo fdiv rc=$?; cat gpurun_out/fdiv_exhaust2.txt
bash tools/llvm_repro/run.sh > gpurun_out/llvm_repro.txt 2>&1; cat gpurun_out/llvm_repro.txt
TAG=cr9 VARIANTS="cr9 fdiv7" CFGS="3 5" REPS=2 bash tools/variant_ab.sh
