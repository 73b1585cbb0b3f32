# Host-side AddressSanitizer pass (device code is not instrumented: the
# sanitizer flags go after -Xarch_host). Builds build/asan/libhec.so and an
# ASan C client of the C ABI, runs the CPU test suite against the ASan library
# here, and prints the GPU-box command for the client's gpu mode.
set -e
cd "$(dirname "$0")/.."
ASANRT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
mkdir -p build/asan
for f in helyim_amd/csrc/*.cpp helyim_amd/csrc/*.hip; do
  x=""; case $f in *.cpp) x="-x hip";; esac
  /opt/rocm/bin/hipcc -O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address \
      -Xarch_host -fno-omit-frame-pointer $x -c $f -o build/asan/$(basename $f).o &
done
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -Xarch_host -fsanitize=address -shared-libasan \
    -o build/asan/libhec.so build/asan/*.o -lpthread
/opt/rocm/lib/llvm/bin/clang -std=c99 -O1 -g -fsanitize=address -shared-libasan tests/c/abi_client.c -Iinclude \
    -Lbuild/asan -lhec -Loracle/build -loracle \
    -Wl,-rpath,$PWD/build/asan:$PWD/oracle/build:$(dirname $ASANRT) -o build/asan/abi_client
HEC_LIB_PATH=$PWD/build/asan/libhec.so LD_PRELOAD=$ASANRT ASAN_OPTIONS=detect_leaks=0 \
    python -m pytest tests -q -m "not gpu" -p no:cacheprovider
ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 ./build/asan/abi_client nogpu
echo "GPU box: ASAN_OPTIONS=detect_leaks=0:verify_asan_link_order=0 ./build/asan/abi_client gpu \$(mktemp -d)"
