set -o pipefail
cd /root/repo
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/variant_parity.py base= rcpn=-DSRBD_RCP_NEWTON > gpurun_out/var_parity.txt 2>&1 && \
timeout -k 10 600 python -u scripts/variant_bench.py --rounds 3 base= rcpn="-DSRBD_RCP_NEWTON" chainp="-DSRBD_CHAIN_PRIO -DSRBD_PROGRESS_PRIO=0" > gpurun_out/var_N10.txt 2>&1 && \
timeout -k 10 600 python -u scripts/variant_bench.py --rounds 3 --horizon 20 base= rcpn="-DSRBD_RCP_NEWTON" > gpurun_out/var_N20.txt 2>&1
