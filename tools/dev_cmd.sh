# development GPU call: the WIP LDS tail search (tools/wip/tail_lds.patch) applied and built on the
# box into a separate library, then its deflate parity and C3/C5 timings against the default
export TMPDIR=/tmp; mkdir -p gpurun_out
rm -rf /tmp/sdzwip && mkdir -p /tmp/sdzwip && cp -r sd-zlib_amd include /tmp/sdzwip/ && (cd /tmp/sdzwip && patch -s -p1 < $OLDPWD/tools/wip/tail_lds.patch && rm -rf sd-zlib_amd/build sd-zlib_amd/lib && timeout -k 10 400 make -s -j16 -C sd-zlib_amd > /dev/null 2>&1) || { echo build-failed; exit 1; }
WIP=/tmp/sdzwip/sd-zlib_amd/lib/libsdz.so
SDZ_LIB=$WIP SDZ_TAIL_LDS=1 timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_deflate_stream.py tests/test_gpu_dict.py -x -q --timeout 240 --timeout-method thread -k "deflate or dict" > gpurun_out/pt_dev1.log 2>&1; rc=$?; tail -1 gpurun_out/pt_dev1.log
for t in 0 1; do
  SDZ_LIB=$WIP SDZ_TAIL_LDS=$t timeout -k 10 120 python3 tools/run_c2.py --mode deflate --steps 2 2>&1 | grep step | tail -1 | sed "s/^/tail_lds=$t C3 /"
  SDZ_LIB=$WIP SDZ_TAIL_LDS=$t timeout -k 10 300 python3 tools/run_configs.py --config c5 2>/dev/null | grep -o '"deflate_kernel_ms": [0-9.]*\|"parity": [a-z]*' | tr '\n' ' ' ; echo " tail_lds=$t C5"
done
exit $rc
