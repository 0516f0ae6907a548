"""The compact fill layout's line index (include/shd_route.h shd_route_tri16_line, used by
the engine's pack kernel and the front end's getters) against its definition: row i's
first 64-byte line = sum over r < i of ceil((na - r) / 6).  CPU only (gcc)."""
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r'''
#include <stdio.h>
#include <stdlib.h>
#include "shd_route.h"
int main(int argc, char** argv) {
    for (int a = 1; a < argc; a++) {
        const int na = atoi(argv[a]);
        for (int i = 0; i <= na; i++) printf("%lld ", (long long)shd_route_tri16_line(na, i));
        printf("\n");
    }
    return 0;
}
'''


def test_tri16_line_matches_definition(tmp_path):
    c = tmp_path / "t.c"
    c.write_text(SRC)
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-O1", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    sizes = [1, 2, 5, 6, 7, 11, 12, 13, 97, 1000, 9337]
    out = subprocess.run([str(exe)] + [str(x) for x in sizes], capture_output=True, text=True, check=True).stdout
    for na, line in zip(sizes, out.strip().splitlines()):
        got = np.array([int(x) for x in line.split()], np.int64)
        want = np.concatenate([[0], np.cumsum([(na - r + 5) // 6 for r in range(na)])])
        assert np.array_equal(got, want), na
    # C4 scale (50,000 attached vertices): the total in lines, 64 B each
    out = subprocess.run([str(exe), "50000"], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[-1]) == sum((50000 - r + 5) // 6 for r in range(50000))
