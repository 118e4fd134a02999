#!/bin/bash
# Run a command in the background; after $1 seconds record GPU utilisation and the kernel wait
# channel of every thread (non-invasive: /proc only), then stop it.
DELAY=$1; shift
OUT=${GRAFT_REPO_ROOT:-.}/gpurun_out/stall
mkdir -p "$OUT"
"$@" > "$OUT/run.log" 2>&1 &
PID=$!
sleep "$DELAY"
if kill -0 $PID 2>/dev/null; then
  echo "still running after ${DELAY}s" > "$OUT/probe.txt"
  (rocm-smi --showuse --showmemuse 2>&1 | grep -v "^$" ) >> "$OUT/probe.txt"
  for t in /proc/$PID/task/*; do
    echo "$(basename $t) $(cat $t/comm) wchan=$(cat $t/wchan 2>/dev/null) syscall=$(cut -d' ' -f1 $t/syscall 2>/dev/null)" >> "$OUT/probe.txt"
  done
  sleep 5
  (rocm-smi --showuse 2>&1 | grep -i "use") >> "$OUT/probe.txt"
  kill $PID; sleep 3; kill -9 $PID 2>/dev/null
  wait $PID
  exit 124
fi
wait $PID
