"""CPU: the Julia `ccall` binding (julia/SCSOptAMD.jl) against the C ABI (include/scsopt.h).

Julia is absent here and on the GPU box, so the binding is never executed; this test pins what
can be checked without it: every `ccall((:scs_*, lib), Ret, (Args...), ...)` names a function the
header declares, with the same number of arguments and Julia types that match the C prototype
(Ptr{Float64} <-> double*, Int64 <-> int64_t, Cint <-> int, Ref{T} <-> T*, Ptr{Cvoid} <-> any
pointer, the 7-pointer scs_history struct as Ref{NTuple{7,Ptr{Float64}}}), and that the binding
reads the IndBox smoothers' bounds the way the reference builds them (closure captures,
phuber-smooth.jl:59-65), not from fields the reference structs do not have.
"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
JL = os.path.join(ROOT, "selfconcordantsmoothoptimization.jl_amd", "julia", "SCSOptAMD.jl")
HDR = os.path.join(ROOT, "include", "scsopt.h")


def _split_top(s, sep=","):
    out, depth, cur = [], 0, ""
    for ch in s:
        if ch in "({[":
            depth += 1
        elif ch in ")}]":
            depth -= 1
        if ch == sep and depth == 0:
            out.append(cur.strip())
            cur = ""
        else:
            cur += ch
    if cur.strip():
        out.append(cur.strip())
    return out


def _header_protos():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"(const char\s*\*|int)\s+(scs_\w+)\s*\(([^;]*?)\)\s*;", src, flags=re.S):
        ret, name, args = m.group(1), m.group(2), " ".join(m.group(3).split())
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        types = []
        for p in params:
            p = re.sub(r"\s*\w+\s*\[\d+\]$", " *", p)          # T id[128] -> T *
            p = re.sub(r"\b\w+\s*(\*?)$", r"\1", p) if not p.endswith("*") else p
            types.append(" ".join(p.replace("*", " * ").split()))
        protos[name] = (ret.replace(" ", ""), types)
    return protos


def _julia_ccalls():
    src = open(JL).read()
    calls = []
    for m in re.finditer(r"ccall\(\(:(\w+),\s*lib\),", src):
        i = m.end()
        depth, j = 1, i
        while depth:
            if src[j] == "(":
                depth += 1
            elif src[j] == ")":
                depth -= 1
            j += 1
        parts = _split_top(src[i:j - 1])
        ret, argt = parts[0], parts[1]
        assert argt.startswith("(") and argt.endswith(")"), (m.group(1), argt)
        inner = argt[1:-1].strip().rstrip(",")
        calls.append((m.group(1), ret, _split_top(inner) if inner else []))
    return calls


C_SCALARS = {"Cint": {"int"}, "Int64": {"int64_t"}, "Float64": {"double"}, "UInt64": {"uint64_t"}, "Csize_t": {"size_t"},
             "Cuint": {"unsigned"}, "Int32": {"int32_t"}}
C_POINTEE = {"Float64": "double", "Int64": "int64_t", "Int32": "int32_t", "Cint": "int", "UInt8": "unsigned char",
             "Cchar": "char"}


def _compatible(jt, ct):
    ct_base = ct.replace("const ", "").strip()
    if ct_base in ("scs_allreduce_fn", "scs_loss_fn"):   # function pointer typedefs (a @cfunction)
        return jt == "Ptr{Cvoid}"
    is_ptr = ct_base.endswith("*")
    if jt in C_SCALARS:
        return (not is_ptr) and ct_base in C_SCALARS[jt]
    if not is_ptr:
        return False
    pointee = ct_base[:-1].strip()
    m = re.fullmatch(r"(Ptr|Ref)\{(.+)\}", jt)
    if not m:
        return False
    inner = m.group(2)
    if inner == "Cvoid":
        return True                                   # void* / scs_ctx* / struct pointers
    if inner == "Ptr{Cvoid}":
        return pointee.endswith("*")                  # scs_ctx** / void**
    if inner.startswith("NTuple{7,Ptr{Float64}}"):
        return pointee == "scs_history"
    return C_POINTEE.get(inner) == pointee


def test_every_ccall_matches_the_header():
    protos = _header_protos()
    calls = _julia_ccalls()
    assert len(calls) >= 15
    seen = set()
    for name, ret, args in calls:
        assert name in protos, f"{name} is not declared in scsopt.h"
        cret, ctypes = protos[name]
        assert (ret == "Cstring") == (cret == "constchar*"), (name, ret, cret)
        assert len(args) == len(ctypes), (name, args, ctypes)
        for a, ct in zip(args, ctypes):
            assert _compatible(a, ct), (name, a, ct)
        seen.add(name)
    # the binding covers the step / loop / comm / sparse entry points a maintainer needs
    for need in ("scs_create", "scs_set_data", "scs_set_sparse", "scs_set_loss", "scs_set_reg", "scs_set_smoother",
                 "scs_method_init", "scs_step_grad", "scs_iterate_ex", "scs_set_comm", "scs_set_reduce_buffer",
                 "scs_reduce_buffer_size", "scs_eval_f"):
        assert need in seen, need


def test_indbox_bounds_come_from_the_closures():
    src = open(JL).read()
    assert "hμ.lb" not in src and "hμ.ub" not in src        # no such fields (phuber-smooth.jl:38-58)
    assert "getfield(g, :lb)" in src and "getfield(g, :ub)" in src
    assert "is_interval_set" in src                         # C_set forms of prox-operators.jl:34-46


def test_callback_user_pointer_is_a_mutable_object():
    """pointer_from_objref throws on immutable objects: the struct whose address libscsopt hands
    back to the loss trampoline must be mutable (and rooted by the model)."""
    src = open(JL).read()
    assert re.search(r"^mutable struct LossCallbacks", src, flags=re.M)
    assert "pointer_from_objref(cbs)" in src and "model.grad_fx = cbs" in src


def test_step_passes_grad_fx():
    """step!(...; ∇fx) reaches the library (scs_step_grad), it is not dropped."""
    src = open(JL).read()
    body = src[src.index("function step!("):]
    body = body[:body.index("\nend")]
    assert "∇fx" in body and "scs_step_grad" in body and ":scs_step," not in body


def _struct_fields(src, name):
    m = re.search(r"mutable struct " + name + r"\b[^\n]*\n(.*?)\nend", src, flags=re.S)
    assert m, name
    body = re.sub(r"#[^\n]*", "", m.group(1))
    return [f.split("::")[0].strip() for f in re.split(r"[;\n]", body) for f in [f] if f.strip()
            for f in f.split(";") if f.strip()]


def test_integration_doc_matches_module():
    """INTEGRATION.md's inline binding is the module's, not an older sketch: the same DeviceProblem
    fields in the same order, and every ccall tuple in the document matches the header too."""
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    mod = open(JL).read()
    fd = [x for f in _struct_fields(doc, "DeviceProblem") for x in f.split() if x]
    fm = [x for f in _struct_fields(mod, "DeviceProblem") for x in f.split() if x]
    assert fd == fm and len(fm) == 19, (fd, fm)
    protos = _header_protos()
    n = 0
    for m in re.finditer(r"ccall\(\(:(\w+),\s*lib\),\s*(\w+),\s*\(([^()]*(?:\{[^{}]*\}[^()]*)*)\)", doc):
        name, ret = m.group(1), m.group(2)
        args = _split_top(m.group(3))
        assert name in protos, name
        cret, ctypes = protos[name]
        assert len(args) == len(ctypes), (name, args, ctypes)
        for a, ct in zip(args, ctypes):
            assert _compatible(a, ct), (name, a, ct)
        n += 1
    assert n >= 5


def test_ggn_grad_fx_one_argument_request():
    """the trampoline answers SCS_CB_GRAD_X (5) by calling grad_fx(x) with x
    alone when applicable (prox-GGN-SCORE.jl:58-59), else stores Julia's own MethodError and returns
    SCS_CB_NO_METHOD (2); chk rethrows a stored callback exception instead of a text error."""
    src = open(JL).read()
    hdr = open(os.path.join(ROOT, "include", "scsopt.h")).read()
    assert re.search(r"#define SCS_CB_GRAD_X 5\b", hdr) and re.search(r"#define SCS_CB_NO_METHOD 2\b", hdr)
    tr = src[src.index("function loss_trampoline("):]
    tr = tr[:tr.index("\nend\n")]
    assert "what == 5" in tr and "applicable(cbs.grad_fx, x)" in tr
    assert "MethodError(cbs.grad_fx, (x,))" in tr and "return Cint(2)" in tr
    assert "cbs.grad_fx(x)" in tr
    ck = src[src.index("function chk("):]
    ck = ck[:ck.index("\nend\n")]
    assert "CB_EXCEPTION[]" in ck and "throw(err)" in ck
