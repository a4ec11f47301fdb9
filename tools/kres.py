"""Per-kernel VGPR / spill counts of a built HIP object (its gfx950 code object's
metadata notes): python tools/kres.py [obj] [name-filter] [--diff other.o]."""
import re
import subprocess
import sys
import tempfile

B = '/opt/rocm/lib/llvm/bin'


def res(obj):
    with tempfile.TemporaryDirectory() as d:
        subprocess.run([B + '/llvm-objcopy', '--dump-section=.hip_fatbin=%s/f' % d, obj], check=True)
        subprocess.run([B + '/clang-offload-bundler', '--unbundle', '--type=o', '--input=%s/f' % d,
                        '--targets=hipv4-amdgcn-amd-amdhsa--gfx950', '--output=%s/co' % d], check=True)
        t = subprocess.run([B + '/llvm-readelf', '--notes', '%s/co' % d], capture_output=True, text=True).stdout
    out = {}
    for b in t.split('  - .agpr_count')[1:]:
        g = lambda k: re.search(r'\.%s:\s+(\S+)' % k, b).group(1)
        out[g('name')] = (int(g('vgpr_count')), int(g('vgpr_spill_count')), int(g('private_segment_fixed_size')),
                          int(g('group_segment_fixed_size')))
    return out


if __name__ == '__main__':
    args = [a for a in sys.argv[1:] if not a.startswith('--')]
    obj = args[0] if args else 'tcpreplay_amd/csrc/build/tcpedit_kernels.o'
    flt = args[1] if len(args) > 1 else ''
    r = res(obj)
    other = res(sys.argv[sys.argv.index('--diff') + 1]) if '--diff' in sys.argv else None
    for k in sorted(r):
        if flt in k and (other is None or other.get(k) != r[k]):
            print(k[:80], 'vgpr %d spill %d priv %d lds %d' % r[k], ('was %s' % (other.get(k),)) if other else '')
