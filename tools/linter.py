"""Lint / auto-format Python sources (reference ``tools/linter.py``).

    python tools/linter.py [PATH ...] [--check]

Uses autopep8 when installed (as the reference did); otherwise falls back to
a dependency-free check: every file must compile and stay within the
project's 100-column limit with no trailing whitespace or tabs.
"""
import argparse
import os
import py_compile
import subprocess
import sys

MAX_COLS = 100
_SKIP = {"__pycache__", ".git", "build", "gpurun_out"}


def python_files(path):
    if os.path.isfile(path):
        yield path
        return
    for root, dirs, files in os.walk(path):
        dirs[:] = sorted(d for d in dirs if d not in _SKIP)
        for f in sorted(files):
            if f.endswith(".py"):
                yield os.path.join(root, f)


def check_file(path):
    problems = []
    try:
        py_compile.compile(path, doraise=True)
    except py_compile.PyCompileError as e:
        return [f"{path}: {e.msg}"]
    with open(path, encoding="utf-8") as f:
        for i, line in enumerate(f, 1):
            line = line.rstrip("\n")
            if len(line) > MAX_COLS:
                problems.append(f"{path}:{i}: line longer than {MAX_COLS} columns")
            if line != line.rstrip():
                problems.append(f"{path}:{i}: trailing whitespace")
            if "\t" in line[:len(line) - len(line.lstrip())]:
                problems.append(f"{path}:{i}: tab indentation")
    return problems


def recursively_lint_files(paths, check_only=False):
    files = [f for p in paths for f in python_files(p)]
    try:
        import autopep8  # noqa: F401
        have_autopep8 = True
    except ImportError:
        have_autopep8 = False
    if have_autopep8 and not check_only:
        subprocess.check_call([sys.executable, "-m", "autopep8", "--max-line-length",
                               str(MAX_COLS), "--in-place"] + files)
    problems = [p for f in files for p in check_file(f)]
    for p in problems:
        print(p)
    print(f"linted {len(files)} files, {len(problems)} problems")
    return problems


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("paths", nargs="*", default=["."])
    ap.add_argument("--check", action="store_true", help="report only, never rewrite")
    a = ap.parse_args(argv)
    return 1 if recursively_lint_files(a.paths, a.check) else 0


if __name__ == "__main__":
    sys.exit(main())
