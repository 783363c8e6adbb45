# run_step SECONDS LOG cmd...: one bounded GPU step; a test / script failure (exit 1) lets the call
# go on, anything else (timeout 124/137, abort 134, segfault 139) or a GPU fault in the log stops it
run_step() {
  local t=$1 log=$2; shift 2
  timeout -k 10 "$t" "$@" > "$log" 2>&1
  local rc=$?
  if grep -qE "Memory access fault|illegal memory access|hipErrorIllegalAddress|HSA_STATUS_ERROR|GPU Hang|page fault" "$log"; then
    echo "GPU fault in $log (rc $rc): stopping"; exit 99
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step $log rc $rc: stopping"; exit $rc; fi
  echo "step $log rc $rc"
  return 0
}
