"""Every `profiles/...` path cited in the docs, sources and tools resolves to a tracked file
(VERDICT r04 item 6).  usage: python tools/check_citations.py  (exit 1 and a list when one does not)"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PAT = re.compile(r"profiles/([A-Za-z0-9_.*\-]+)")


def main():
    files = subprocess.run(["git", "ls-files"], cwd=ROOT, capture_output=True, text=True, check=True).stdout.split()
    tracked = set(files)
    scan = [f for f in files if f.endswith((".md", ".py", ".hip", ".hpp", ".h", ".sh", ".c"))
            and not f.startswith(("profiles/", "tools/sessions")) and f not in ("VERDICT.md", "ADVICE.md")]
    bad = []
    for f in scan:
        for n, line in enumerate(open(os.path.join(ROOT, f), errors="replace"), 1):
            for m in PAT.finditer(line):
                name = m.group(1).rstrip(".,;:)`")
                if not name or "*" in name or "<" in name or name.endswith("_") or "{" in name:
                    continue   # a pattern, not a file
                if f"profiles/{name}" not in tracked:
                    bad.append(f"{f}:{n}: profiles/{name}")
    for b in bad:
        print(b)
    print(f"{len(bad)} unresolved citation(s)")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
