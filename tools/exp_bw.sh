set -e; timeout -k 10 200 ./tools/bw_probe 134217728 0 > gpurun_out/bw0.txt 2>&1; timeout -k 10 200 ./tools/bw_probe 134217728 256 > gpurun_out/bw256.txt 2>&1
