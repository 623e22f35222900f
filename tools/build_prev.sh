# build the library of git HEAD (or $1) into rust-simd-r-drive_amd/build/var/lib_prev.so (same-box A/Bs)
set -e
rev=${1:-HEAD}
rm -rf /tmp/prevwt
git worktree add -f /tmp/prevwt $rev >/dev/null 2>&1
make -C /tmp/prevwt/rust-simd-r-drive_amd >/dev/null 2>&1
mkdir -p rust-simd-r-drive_amd/build/var
cp /tmp/prevwt/rust-simd-r-drive_amd/build/libsrd_amd.so rust-simd-r-drive_amd/build/var/lib_prev.so
git worktree remove --force /tmp/prevwt
