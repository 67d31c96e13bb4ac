# dev: one GPU call of variant timings (tools/variant_bench.py); output in gpurun_out/var.log
set -u
L=raysnail_amd/lib
V="timeout -k 10 300 python -u tools/variant_bench.py"
{ $V --scene=c4 $L/libraysnail_hip.so $L/var_regen.so && $V --scene=rtow $L/libraysnail_hip.so $L/var_regen.so && $V --scene=quadric $L/libraysnail_hip.so $L/var_regen.so; } > gpurun_out/var.log 2>&1
