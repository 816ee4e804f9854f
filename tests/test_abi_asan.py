"""CPU: the C ABI's host side under AddressSanitizer: a host-only ASAN build of
libonetrans_hip (make -C recommend_amd/csrc asan: --offload-host-only, no device code) linked into
tests/abi_asan_check.c (compiled by the ROCm clang, whose ASAN runtime the library's
instrumentation expects), which drives every checked entry point down its argument-validation error path
and the workspace-size queries at edge sizes.  No GPU is touched (the calls return before any launch)."""

import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'recommend_amd', 'csrc')
ASAN_DIR = os.path.join(ROOT, 'build', 'asan')
LIB = os.path.join(ASAN_DIR, 'libonetrans_hip_asan.so')


@pytest.mark.skipif(not os.path.exists('/opt/rocm/bin/hipcc') or not os.path.exists('/opt/rocm/lib/llvm/bin/clang'),
                    reason='needs hipcc and the ROCm clang (the ASAN runtime must match hipcc\'s)')
def test_abi_error_paths_under_asan(tmp_path):
    jobs = str(min(8, os.cpu_count() or 4))
    subprocess.run(['make', '-C', CSRC, '-j', jobs, 'asan', f'ASAN_DIR={ASAN_DIR}'], check=True,
                   stdout=subprocess.PIPE, stderr=subprocess.STDOUT, timeout=600)
    exe = str(tmp_path / 'abi_asan_check')
    subprocess.run(['/opt/rocm/lib/llvm/bin/clang', '-fsanitize=address', '-g', '-I', os.path.join(ROOT, 'include'),
                    os.path.join(ROOT, 'tests', 'abi_asan_check.c'), '-o', exe, '-L', ASAN_DIR,
                    '-lonetrans_hip_asan', f'-Wl,-rpath,{ASAN_DIR}', '-L/opt/rocm/lib', '-lamdhip64',
                    '-Wl,-rpath,/opt/rocm/lib'], check=True, timeout=120)
    env = dict(os.environ, ASAN_OPTIONS='detect_leaks=0:abort_on_error=0', HIP_VISIBLE_DEVICES='')
    r = subprocess.run([exe], stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env, timeout=120)
    out = r.stdout.decode(errors='replace')
    assert 'AddressSanitizer' not in out, out
    assert r.returncode == 0 and 'ABI ASAN CHECK OK' in out, out
