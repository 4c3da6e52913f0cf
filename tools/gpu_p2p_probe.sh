# two processes on the one GPU: IPC-mapped mailbox ping-pong (kernel stores / stream write+wait value)
set -e
O=gpurun_out/p2p
mkdir -p $O
D=$(mktemp -d)
timeout -k 5 60 ./tools/p2p_probe 0 $D 2000 > $O/r0.json 2> $O/r0.err &
P0=$!
timeout -k 5 60 ./tools/p2p_probe 1 $D 2000 > $O/r1.json 2> $O/r1.err
R1=$?
wait $P0
R0=$?
rm -rf $D
echo "rc $R0 $R1" > $O/rc.txt
