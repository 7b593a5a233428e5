#!/usr/bin/env python3
"""Copy include/vpt_run.hpp verbatim into INTEGRATION.md §1's code block (tests/test_gpu_integration.py checks
that the two agree)."""
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
doc = (ROOT / "INTEGRATION.md").read_text()
src = (ROOT / "include" / "vpt_run.hpp").read_text().strip()
start = doc.index("```cpp\n// vpt_run.hpp")
end = doc.index("\n```", start + 7)
(ROOT / "INTEGRATION.md").write_text(doc[:start] + "```cpp\n" + src + doc[end:])
print("INTEGRATION.md §1 <- include/vpt_run.hpp")
