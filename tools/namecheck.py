"""Names read in a module that nothing in it defines (a cheap stand-in for pyflakes, which the image
lacks): catches a helper deleted by an edit in code paths the CPU suite cannot execute (the GPU
dispatch). usage: namecheck.py file.py ... ; exit 1 and the names if any."""
import ast
import builtins
import sys


def undefined(src: str) -> set:
    t = ast.parse(src)
    defined = set(dir(builtins)) | {"__file__", "__name__", "__doc__"}
    for n in ast.walk(t):
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            defined.add(n.name)
        elif isinstance(n, ast.Import):
            defined.update(a.asname or a.name.split(".")[0] for a in n.names)
        elif isinstance(n, ast.ImportFrom):
            defined.update(a.asname or a.name for a in n.names)
        elif isinstance(n, ast.arg):
            defined.add(n.arg)
        elif isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            defined.add(n.id)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            defined.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            defined.update(n.names)
    used = {n.id for n in ast.walk(t) if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load)}
    return used - defined


if __name__ == "__main__":
    bad = 0
    for f in sys.argv[1:]:
        u = undefined(open(f).read())
        if u:
            print(f, sorted(u))
            bad = 1
    sys.exit(bad)
