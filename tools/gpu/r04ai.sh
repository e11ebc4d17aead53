# round 4: decode phase stamps, containertest (packed subroutine areas) and vecrec
mkdir -p gpurun_out/r04ai
timeout -k 10 300 python -u tools/tune/enc_stamps.py run containertest vecrec > gpurun_out/r04ai/stamps.log 2>&1 || exit 1
