cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 python -u tools/mb_table_sync.py > gpurun_out/table_sync.log 2>&1
