set -u
timeout -k 10 60 tools/excp_probe > gpurun_out/excp_probe.txt 2>&1; echo excp rc=$?; cat gpurun_out/excp_probe.txt
timeout -k 10 300 python tools/phase_profile.py 65536 casenml ref as-generated 8 1 > gpurun_out/phase_cfg2.txt 2>&1; echo phase rc=$?; cat gpurun_out/phase_cfg2.txt
