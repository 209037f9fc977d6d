#!/bin/bash
# Round 4 w: the sort changes (4-key-vector chunk histogram, 2048-entry chunks) -- PlonK parity, every
# part rehearsed alone, the roofline record's PMC passes of this tree, the
# driver's bench command, then the full -m gpu suite and smoke.
cd "${GRAFT_REPO_ROOT:-.}"
V=r04w bash tools/gpu_r04o.sh && grep -q done gpurun_out/progress_r04w.txt || exit 2
V=r04w bash tools/gpu_r04p.sh
