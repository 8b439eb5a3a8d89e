# sourced by the tools/gpu_*.sh scripts: `step NAME SECONDS cmd...` runs one GPU step under its own
# time limit, logs to $O/NAME.log, and ends the script on a time limit, abort or segfault (124, 134,
# 137, 139): nothing more is started on the GPU after such a step. Ordinary failures (test asserts,
# rc 1..3) are recorded and the script goes on.
step() {
  local name=$1 secs=$2
  shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" >> "$O/rc.txt"
  case $rc in
    124|134|137|139) echo "stopping after $name (rc $rc)" >> "$O/rc.txt"; exit $rc ;;
  esac
  return 0
}
