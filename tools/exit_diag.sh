# Which native-library usage pattern makes a Python process hang at exit (no torch)?
cd "${GRAFT_REPO_ROOT:-.}"
run() { local name=$1; shift; timeout -k 5 25 "$@" > /dev/null 2>&1; echo "$name rc=$?"; }
run A_count python -c "import ctypes; L=ctypes.CDLL('walkai_nos_amd/_native/libnos_probe.so'); n=ctypes.c_int(); L.nos_probe_device_count(ctypes.byref(n)); print(n.value)"
run B_stream python -c "from walkai_nos_amd.ops import probe as P; s=P.Stream(0, list(range(32))); s.close(); print('ok')"
run C_mfma python -c "from walkai_nos_amd.ops import probe as P; print(P.probe_mfma('fp32', 0, None, iters=64, reps=1))"
run D_mfma_torch python -c "import torch; from walkai_nos_amd.ops import probe as P; print(P.probe_mfma('fp32', 0, None, iters=64, reps=1))"
run E_hbm python -c "from walkai_nos_amd.ops import probe as P; print(P.probe_hbm(0, None, nbytes=1<<24, reps=1))"
