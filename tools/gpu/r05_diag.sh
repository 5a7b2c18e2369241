cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 120 python3 tools/diag_blocks.py product force_reduce_mask=1 force_reduce_mask=0 force_reduce_mask=1 || exit 1
