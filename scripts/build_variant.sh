# Build libgmp.so + libgmp_torch.so of a git revision (default HEAD) into abvar/NAME/ for A/B runs
# on the GPU box: GMP_LIB=abvar/NAME/libgmp.so GMP_TORCH_LIB=abvar/NAME/libgmp_torch.so python ...
# (libgmp_torch.so resolves libgmp.so next to itself).  usage: build_variant.sh NAME [REV]
set -e
NAME=$1; REV=${2:-HEAD}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=/tmp/gmp_var_$NAME
rm -rf "$TMP" && mkdir -p "$TMP"
git -C "$ROOT" archive "$REV" geometric-message-passing_amd/csrc include | tar -x -C "$TMP"
mkdir -p "$TMP/geometric-message-passing_amd/gmp_amd"
make -C "$TMP/geometric-message-passing_amd/csrc" -j${JOBS:-8} > "$TMP/build.log" 2>&1
mkdir -p "$ROOT/abvar/$NAME"
cp "$TMP/geometric-message-passing_amd/gmp_amd/libgmp.so" "$TMP/geometric-message-passing_amd/gmp_amd/libgmp_torch.so" "$ROOT/abvar/$NAME/"
echo "built abvar/$NAME from $REV"
