# Round-end check of the final in-tree build: full GPU suite and smoke.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAILN=3 TAG=r04jj bash scripts/gpu_steps.sh \
  '900|pytest|python -u -m pytest tests/ -m gpu -q --timeout 300 --timeout-method thread' \
  '240|smoke|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"'
