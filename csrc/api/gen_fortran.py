"""Generate the Fortran 2003 module (slate_c_api.f90) from c_api.h.

Reference capability: tools/fortran/generate_fortran_module.py, which parses
the reference's C API headers and writes a bind(c) interface per function.
Here the C API is declared once per precision through SLATE_C_API_DECLARE;
this script expands that macro for r32 / r64 / c32 / c64, parses every
prototype, and maps C types onto iso_c_binding kinds:

  handles (slate_Matrix_X, slate_Pivots, ...)  -> type(c_ptr), value
  int / int64_t / uint64_t / float / double   -> integer/real kinds, value
  scalar_t                                    -> real or complex kind, value
  slate_Side / Op / Uplo / Diag / Norm / Target -> character(kind=c_char), value
  T* (data arrays, Lambda, Sigma)             -> assumed-size array T(*)
  int* (iteration count)                      -> integer(c_int) by reference
  const char* (matgen kind)                   -> character(kind=c_char) s(*)
  slate_Options const*                        -> type(slate_Options) opts(*)

usage: python csrc/api/gen_fortran.py [out.f90]   (default: next to this file)
"""
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
HEADER = os.path.join(HERE, "..", "include", "slate_amd", "c_api.h")

PREC = {  # suffix: (scalar kind decl, real kind decl, kind names to import)
    "r32": ("real(c_float)", "real(c_float)", {"c_float"}),
    "r64": ("real(c_double)", "real(c_double)", {"c_double"}),
    "c32": ("complex(c_float_complex)", "real(c_float)", {"c_float_complex", "c_float"}),
    "c64": ("complex(c_double_complex)", "real(c_double)", {"c_double_complex", "c_double"}),
}
CHAR_TYPES = {"slate_Target", "slate_Op", "slate_Uplo", "slate_Diag", "slate_Side", "slate_Norm"}


def strip_comments(s):
    return re.sub(r"/\*.*?\*/", "", s, flags=re.S)


def prototypes(text):
    """Yield 'ret name(args)' strings for every function prototype."""
    text = re.sub(r"\\\n", " ", strip_comments(text))
    for stmt in text.split(";"):
        stmt = " ".join(stmt.split())
        m = re.search(r"([A-Za-z_][\w\s\*]*?)\b(slate_\w+)\s*\(([^()]*)\)\s*$", stmt)
        if m and not stmt.lstrip().startswith(("typedef", "#")):
            yield m.group(1).strip(), m.group(2), m.group(3).strip()


def expand(text):
    """Macro body instantiated per precision + the non-macro prototypes."""
    body = re.search(r"#define SLATE_C_API_DECLARE\(X, scalar_t, real_t\)(.*?)\n\s*\n", text, flags=re.S).group(1)
    out = []
    for x in PREC:
        inst = body.replace("##X##", x).replace("##X", x)
        inst = re.sub(r"\bscalar_t\b", f"__scalar_{x}", inst)
        inst = re.sub(r"\breal_t\b", f"__real_{x}", inst)
        out.append(inst)
    rest = text.replace(body, "")
    return "\n".join(out), rest


def ftype(ctype, name, kinds):
    """Fortran declaration for one C parameter; records the kinds to import."""
    t = ctype.replace("const", "").strip()
    ptr = t.endswith("*")
    t = t.rstrip("*").strip()
    m = re.match(r"__(scalar|real)_(\w+)", t)
    if m:
        sc, re_, ks = PREC[m.group(2)]
        kinds |= ks
        decl = sc if m.group(1) == "scalar" else re_
        return f"{decl} :: {name}(*)" if ptr else f"{decl}, value :: {name}"
    if t.startswith("slate_Options"):
        kinds.add("slate_Options")
        return f"type(slate_Options) :: {name}(*)"
    if t.startswith(("slate_Matrix", "slate_TriangularFactors", "slate_Pivots")):
        kinds.add("c_ptr")
        return f"type(c_ptr), value :: {name}"
    if t in CHAR_TYPES or (t == "char" and not ptr):
        kinds.add("c_char")
        return f"character(kind=c_char), value :: {name}"
    if t == "char" and ptr:
        kinds.add("c_char")
        return f"character(kind=c_char) :: {name}(*)"
    base = {"int": ("integer(c_int)", "c_int"), "int64_t": ("integer(c_int64_t)", "c_int64_t"),
            "uint64_t": ("integer(c_int64_t)", "c_int64_t"), "double": ("real(c_double)", "c_double"),
            "float": ("real(c_float)", "c_float")}[t]
    kinds.add(base[1])
    return f"{base[0]} :: {name}" if ptr else f"{base[0]}, value :: {name}"


def interface(ret, name, args):
    kinds = set()
    params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
    names, decls = [], []
    for p in params:
        m = re.match(r"(.*?)(\w+)$", p)
        ctype, pname = m.group(1).strip(), m.group(2)
        names.append(pname)
        decls.append(ftype(ctype, pname, kinds))
    is_sub = ret.strip() == "void"
    if not is_sub:
        if ret.replace("const", "").strip() == "char*":
            kinds.add("c_ptr")
            rdecl = f"type(c_ptr) :: {name}"
        else:
            rdecl = ftype(ret, name, kinds).replace(", value", "")
    kw = "subroutine" if is_sub else "function"
    lines = [f"        {kw} {name}({', '.join(names)}) &", f"                bind(c, name=\"{name}\")"]
    if kinds:
        lines.append(f"            import :: {', '.join(sorted(kinds))}")
    lines += [f"            {d}" for d in decls]
    if not is_sub:
        lines.append(f"            {rdecl}")
    lines.append(f"        end {kw}")
    return "\n".join(lines)


def options(text):
    return re.findall(r"(slate_Option_\w+)\s*=\s*(\d+)", text)


def main():
    with open(HEADER) as f:
        text = f.read()
    per_prec, rest = expand(text)
    protos = list(prototypes(rest)) + list(prototypes(per_prec))
    seen, ifaces = set(), []
    for ret, name, args in protos:
        if name in seen:
            continue
        seen.add(name)
        ifaces.append(interface(ret, name, args))
    opts = options(text)
    out = ["! GENERATED by csrc/api/gen_fortran.py from csrc/include/slate_amd/c_api.h -- do not edit.",
           "! Fortran 2003 bindings (iso_c_binding) for the whole C API (reference capability:",
           "! the generated Fortran module of tools/fortran/generate_fortran_module.py).",
           "! Handles are type(c_ptr); scalars are passed by value as in c_api.h; data",
           "! arrays are assumed-size, so a 2-D Fortran array can be passed directly.",
           "module slate_amd", "    use iso_c_binding", "    implicit none", "",
           "    type, bind(c) :: slate_Options", "        integer(c_int) :: option",
           "        integer(c_int64_t) :: ivalue", "        real(c_double) :: dvalue",
           "    end type slate_Options", ""]
    out += [f"    integer(c_int), parameter :: {k} = {v}" for k, v in opts]
    out += ["", "    interface"]
    out += ["\n\n".join(ifaces)]
    out += ["    end interface", "end module slate_amd", ""]
    dst = sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "slate_c_api.f90")
    with open(dst, "w") as f:
        f.write("\n".join(out))
    print(f"{dst}: {len(ifaces)} interfaces, {len(opts)} option keys")


if __name__ == "__main__":
    main()
