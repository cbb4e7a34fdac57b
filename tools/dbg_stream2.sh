#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"

MPX_LIB=$PWD/minpaxos_amd/libmpx_dbg.so timeout -k 10 120 python tools/dbg_stream.py 2>&1 | head -40
