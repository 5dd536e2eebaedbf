# Diagnostic libgmp.so builds of the working tree with -DGMP_K7G_DIAG=<bits> (gmp_tpgemm.hip):
# abvar/k7g<bits>/libgmp.so.  usage: build_diag.sh BITS...
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
cd "$ROOT/geometric-message-passing_amd/csrc"
for b in "$@"; do
  mkdir -p build_diag$b "$ROOT/abvar/k7g$b"
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function \
    -munsafe-fp-atomics -DGMP_K7G_DIAG=$b -c gmp_tpgemm.hip -o build_diag$b/gmp_tpgemm.o
  objs=$(ls build/*.o | grep -v gmp_tpgemm.o)
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Wl,-soname,libgmp.so \
    -o "$ROOT/abvar/k7g$b/libgmp.so" $objs build_diag$b/gmp_tpgemm.o
  rm -rf build_diag$b
  echo "built abvar/k7g$b"
done
