# Snapshot the tree into .gpu_frozen/ (git-ignored) so that a queued GPU call runs exactly
# this state while the working tree keeps changing: tracked + untracked-not-ignored files,
# the built libraries and executables, and the reference checkers (mtimes kept, so the
# `built` test fixture finds nothing to rebuild).   usage: bash tools/freeze.sh
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
F=$R/.gpu_frozen
rm -rf "$F"
mkdir -p "$F"
cd "$R"
{ git ls-files --cached --others --exclude-standard; \
  find canu_amd/lib canu_amd/bin oracle/_build -type f 2>/dev/null; \
  find oracle/_ref -maxdepth 1 -type f 2>/dev/null; } | sort -u | tar -cf - -T - | tar -xf - -C "$F"
echo "frozen $(du -sh "$F" | cut -f1) at $(git rev-parse --short HEAD)"
