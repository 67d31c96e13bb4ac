# dev: one GPU call of variant timings (tools/variant_bench.py); output in gpurun_out/var.log
set -u
L=raysnail_amd/lib
V="timeout -k 10 300 python -u tools/variant_bench.py"
{ $V --scene=c4 $L/libraysnail_hip.so $L/var_n2w1.so && $V --scene=rtow $L/var_0base.so $L/libraysnail_hip.so $L/var_0base.so $L/libraysnail_hip.so; } > gpurun_out/var.log 2>&1
