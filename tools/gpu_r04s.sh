#!/bin/bash
# Round 4 s: the fused PlonK ratio (one thread per peer) -- PlonK parity, every
# part rehearsed alone, the roofline record's PMC passes of this tree, the
# driver's bench command, then the full -m gpu suite and smoke.
cd "${GRAFT_REPO_ROOT:-.}"
V=r04s bash tools/gpu_r04o.sh && grep -q done gpurun_out/progress_r04s.txt || exit 2
V=r04s bash tools/gpu_r04p.sh
