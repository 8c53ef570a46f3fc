"""A source invariant of the device code (profiles/r06_hang_isa.txt).

Round 5's region_long_kernel hung the GPU: a value produced inside a lane-0-only branch (`if (lane == 0)
q = atomicAdd(...)`) was broadcast with __builtin_amdgcn_readfirstlane inside a loop. The compiler does
not promise that the wave reconverges before the readfirstlane: it rotated the loop so that lanes 1..63
re-entered it without lane 0 and readfirstlane read their own zero, forever. The fix runs such atomics on
every lane (lane 0 adding, the others adding 0), so the broadcast value never comes out of a lane-0-only
branch. This test keeps the pattern out of the product kernels, and checks that it catches the round-5
source."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ambry_amd", "csrc")

_RFL = re.compile(r"__builtin_amdgcn_readfirstlane\(\s*(?:\([^()]*\)\s*)?([A-Za-z_]\w*)\s*\)")
_LANE0 = re.compile(r"if\s*\(\s*(?:lane\s*==\s*0|!\s*lane|threadIdx\.x\s*==\s*0)\b")


def lane0_broadcasts(text: str, window: int = 16):
    """(line number, variable) of every readfirstlane(v) whose v is assigned inside an `if (lane == 0)` branch
    within the `window` lines before it (a single-statement if, or a braced block)."""
    lines = text.splitlines()
    found = []
    for i, line in enumerate(lines):
        for m in _RFL.finditer(line):
            var = m.group(1)
            assign = re.compile(r"\b%s\s*(?:[-+|^&]?=)(?!=)" % re.escape(var))
            for j in range(max(0, i - window), i):
                if not _LANE0.search(lines[j]):
                    continue
                # the branch: the rest of line j, and a braced block's lines up to its closing brace
                body = [lines[j][_LANE0.search(lines[j]).end():]]
                if lines[j].rstrip().endswith("{"):
                    depth = 1
                    for k in range(j + 1, i):
                        depth += lines[k].count("{") - lines[k].count("}")
                        body.append(lines[k])
                        if depth <= 0:
                            break
                if any(assign.search(b) for b in body):
                    found.append((i + 1, var))
                    break
    return found


def test_no_lane0_value_broadcast_in_product_kernels():
    bad = []
    for name in sorted(os.listdir(CSRC)):
        if name.endswith((".hip", ".h")):
            with open(os.path.join(CSRC, name)) as f:
                bad += [(name, ln, v) for ln, v in lane0_broadcasts(f.read())]
    assert not bad, "readfirstlane of a value set in a lane-0-only branch: %r" % bad


def test_lint_catches_the_round5_claim_loop():
    """The claim loop of round 5's region_long_kernel (b95e535^, message_kernels.hip) and the done count of
    round 6's first form are flagged; their converged forms are not."""
    claim = """
  for (;;) {
    uint32_t q = 0;
    if (lane == 0) q = atomicAdd(g.lng.claim, 1u);
    q = __builtin_amdgcn_readfirstlane(q);
    if (q >= total) break;
  }"""
    done = """
    uint32_t prev = 0;
    if (lane == 0) {
      g.lng.slot[q] = c;
      __threadfence();
      prev = atomicAdd(&lr.done, 1u);
    }
    prev = __builtin_amdgcn_readfirstlane(prev);"""
    listed = """
      bool ok = false;
      if (lane == 0) ok = list_long(*lng, pa, jl, ex, i, record_bit(k));
      if (__builtin_amdgcn_readfirstlane((uint32_t)ok)) continue;"""
    converged = """
    if (lane == 0) g.lng.slot[q] = c;
    __threadfence();
    const uint32_t prev = __builtin_amdgcn_readfirstlane(atomicAdd(&lr.done, lane == 0 ? 1u : 0u));"""
    assert [v for _, v in lane0_broadcasts(claim)] == ["q"]
    assert [v for _, v in lane0_broadcasts(done)] == ["prev"]
    assert [v for _, v in lane0_broadcasts(listed)] == ["ok"]
    assert lane0_broadcasts(converged) == []
