set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/attn_pmc_sq.sh kvA flash_bwd_kv5 "tools/attn_abx.py x /tmp/x" && MSQ_LIB_PATH=_ablib/base.so bash tools/attn_pmc_sq.sh kvB flash_bwd_kv5 "tools/attn_abx.py x /tmp/x"
