set -o pipefail
mkdir -p gpurun_out
uname -r
sysctl net.ipv4.tcp_mem net.ipv4.tcp_wmem net.ipv4.tcp_rmem 2>/dev/null || cat /proc/sys/net/ipv4/tcp_mem
timeout -k 5 100 python tools/socket_floor.py --clients 8 --elems 100000000 --rounds 2 --overlap --client-sequential --sendfile --timeout 60 > gpurun_out/sockprobe1.jsonl 2>&1; echo rc1=$?
cut -c1-400 gpurun_out/sockprobe1.jsonl | tail -3
timeout -k 5 100 python tools/socket_floor.py --clients 8 --elems 100000000 --rounds 2 --overlap --client-sequential --timeout 60 > gpurun_out/sockprobe2.jsonl 2>&1; echo rc2=$?
cut -c1-400 gpurun_out/sockprobe2.jsonl | tail -3
