export TMPDIR=/tmp
O=gpurun_out/r6t; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lds -o t -- python tools/prof_target.py apgstep 2048 200 > $O/lds.log 2>&1 &&
PROF_FORCE_GLOBAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/glb -o t -- python tools/prof_target.py apgstep 2048 200 > $O/glb.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/vjp -o t -- python tools/prof_target.py vjp 2048 256 > $O/vjp.log 2>&1
[ $? -eq 0 ] && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5 -o t -- python tools/c5_update_probe.py 1 > $O/c5.log 2>&1
rc=$?; find $O -name '*_kernel_trace.csv' -delete; exit $rc
