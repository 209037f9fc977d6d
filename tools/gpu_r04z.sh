#!/bin/bash
# Round 4 z: the driver's N > 1 launch shape (torchrun over gloo, ranks sharing
# one GPU) rehearsed again on the final tree (r04_w): tools/gpu_r04g.sh.
cd "${GRAFT_REPO_ROOT:-.}"
V=r04z bash tools/gpu_r04g.sh
