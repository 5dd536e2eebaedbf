# Build the WORKING TREE's libraries with extra compile flags into abvar/NAME/ (A/B of
# compile-time variants): build_tree_variant.sh NAME "-DFOO=1 ..."
set -e
NAME=$1; FLAGS=$2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=/tmp/gmp_tvar_$NAME
rm -rf "$TMP" && mkdir -p "$TMP"
cp -r "$ROOT/geometric-message-passing_amd" "$ROOT/include" "$TMP/"
rm -rf "$TMP/geometric-message-passing_amd/csrc/build"
make -C "$TMP/geometric-message-passing_amd/csrc" -j${JOBS:-8} \
  CXXFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function -munsafe-fp-atomics $FLAGS" \
  > "$TMP/build.log" 2>&1
mkdir -p "$ROOT/abvar/$NAME"
cp "$TMP/geometric-message-passing_amd/gmp_amd/libgmp.so" "$TMP/geometric-message-passing_amd/gmp_amd/libgmp_torch.so" "$ROOT/abvar/$NAME/"
echo "built abvar/$NAME ($FLAGS)"
