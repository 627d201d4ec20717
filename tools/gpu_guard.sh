# Source me.  run <limit_s> <cmd...>: runs one GPU step under its own time limit;
# stops the whole script after a time-out, abort or fault, continues after an
# ordinary failure (e.g. an unknown counter name).
run() {
    local lim=$1; shift
    timeout -k 10 "$lim" "$@"
    local rc=$?
    echo "[step rc=$rc] $*" >&2
    case $rc in
        124|137|134|139|135|132) echo "[guard] fatal rc=$rc, stopping" >&2; exit $rc;;
    esac
    return 0
}
