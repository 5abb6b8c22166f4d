"""A small interpreter for the subset of MATLAB the reference's hot path is written in.

Test infrastructure only (tests/golden/make_ref_golden.py): it reads the reference's own .m files at
generation time -- main.m, functions/ReadFiles.m, findSetting.m, Buildxhat.m, BuildAwG.m, BuildRSD.m,
sumabs.m -- and executes their statements with MATLAB's value semantics in IEEE double precision, so
the committed fixtures are the numbers the reference's text produces, not those of a restatement.
Nothing of the .m text is stored; only the numbers the run produces are.

How it works: a tokenizer (MATLAB's context rules: transpose vs quote, whitespace as element separator
inside [] and {} literals, command syntax), a recursive-descent parser to an AST, and a compiler from
the AST to Python source that calls the runtime below (m_* functions: column-major indexing with
growth, cs-lists, cells, struct arrays, string arrays, implicit expansion, matrix vs element-wise
operators).  A name is a variable if the function assigns it anywhere, otherwise a function call --
the rule MATLAB applies to the code at hand.  Long scalar expressions (the generated Jacobian terms of
BuildAwG.m) get a second, plain-float Python form guarded by an all-operands-are-doubles check, which
makes a cam0 iteration take seconds.

The MATLAB built-ins the text calls are restated here (size, zeros, strcmp, str2double, unique, diag,
repmat, inv via ^-1, readmatrix with the options ReadFiles.m passes, dir, fileparts, ...): they are
library functions, not reference code.  Matrix inverse and products go to numpy's LAPACK / BLAS
(MATLAB's go to MKL): the same algorithms, rounding-level differences.
"""
import copy
import fnmatch
import math
import os
import re

import numpy as np

# ----------------------------------------------------------------------------------------------
# values
# ----------------------------------------------------------------------------------------------


class _Undef:
    def __repr__(self):
        return "UNDEF"


UNDEF = _Undef()
COLON = ":"


class MatlabError(Exception):
    pass


class MainReturn(Exception):
    pass


def EMPTY():
    return np.zeros((0, 0))


class CSList(list):
    """a comma-separated list (c{:}, s.field of a struct array)"""


class MCell:
    __slots__ = ("a",)

    def __init__(self, a):
        self.a = a  # 2-D object ndarray

    @staticmethod
    def empty(r, c):
        a = np.empty((r, c), dtype=object)
        for i in range(r):
            for j in range(c):
                a[i, j] = EMPTY()
        return MCell(a)

    @property
    def shape(self):
        return self.a.shape

    def __deepcopy__(self, memo):
        b = np.empty(self.a.shape, dtype=object)
        for idx in np.ndindex(self.a.shape):
            b[idx] = copy.deepcopy(self.a[idx], memo)
        return MCell(b)

    def __repr__(self):
        return f"MCell{self.a.shape}"


class MStr:
    """MATLAB string array (None = <missing>)"""
    __slots__ = ("a",)

    def __init__(self, a):
        self.a = a

    @staticmethod
    def scalar(s):
        a = np.empty((1, 1), dtype=object)
        a[0, 0] = s
        return MStr(a)

    @property
    def shape(self):
        return self.a.shape

    def __deepcopy__(self, memo):
        return MStr(self.a.copy())

    def __repr__(self):
        return f"MStr{self.a.shape}"


class MStruct:
    """struct array, 1 x n (a scalar struct is 1 x 1)"""
    __slots__ = ("elems", "fields")

    def __init__(self, elems=None, fields=None):
        self.elems = [{}] if elems is None else elems
        self.fields = list(fields) if fields is not None else []
        for e in self.elems:
            for k in e:
                if k not in self.fields:
                    self.fields.append(k)

    @property
    def shape(self):
        return (1, len(self.elems)) if self.elems else (0, 0)

    def get(self, k, name):
        e = self.elems[k]
        if name in e:
            return e[name]
        if name in self.fields:
            return EMPTY()
        raise MatlabError(f"Reference to non-existent field '{name}'")

    def __deepcopy__(self, memo):
        return MStruct([{k: copy.deepcopy(v, memo) for k, v in e.items()} for e in self.elems], self.fields)

    def __repr__(self):
        return f"MStruct(1x{len(self.elems)}: {self.fields})"


class FuncHandle:
    def __init__(self, name):
        self.name = name


def m_cp(x):
    """value semantics on plain assignment (x = y)"""
    if isinstance(x, (np.ndarray, MCell, MStruct, MStr)):
        return copy.deepcopy(x)
    return x


def is_text(x):
    return isinstance(x, str) or (isinstance(x, MStr) and x.a.size == 1)


def text_of(x):
    if isinstance(x, str):
        return x
    if isinstance(x, MStr):
        return x.a.flat[0]
    raise MatlabError(f"not text: {x!r}")


def shape_of(x):
    if isinstance(x, (float, int, bool, np.floating, np.integer, np.bool_)):
        return (1, 1)
    if isinstance(x, str):
        return (1, len(x)) if x else (0, 0)
    if isinstance(x, np.ndarray):
        return x.shape
    if isinstance(x, (MCell, MStr, MStruct)):
        return x.shape
    if isinstance(x, FuncHandle):
        return (1, 1)
    raise MatlabError(f"size of {x!r}")


def numel(x):
    r, c = shape_of(x)
    return r * c


def scal(x):
    """numeric 1x1 -> python float (bool stays bool)"""
    if isinstance(x, np.ndarray):
        if x.size != 1:
            return x
        v = x.flat[0]
        if x.dtype == bool:
            return bool(v)
        return float(v)
    if isinstance(x, np.floating):
        return float(x)
    if isinstance(x, np.bool_):
        return bool(x)
    return x


def arr(x):
    """numeric value -> 2-D ndarray"""
    if isinstance(x, np.ndarray):
        return x if x.ndim == 2 else x.reshape(1, -1) if x.ndim == 1 else x.reshape(1, 1)
    if isinstance(x, bool):
        return np.array([[x]])
    if isinstance(x, (float, int, np.floating, np.integer, np.bool_)):
        return np.array([[float(x)]])
    if isinstance(x, str):
        return np.array([[float(ord(ch)) for ch in x]]) if x else np.zeros((0, 0))
    raise MatlabError(f"not numeric: {x!r}")


def m_true(x):
    if isinstance(x, bool):
        return x
    if isinstance(x, (float, int, np.floating, np.integer, np.bool_)):
        return x != 0
    if isinstance(x, np.ndarray):
        return x.size > 0 and bool(np.all(x != 0))
    if isinstance(x, str):
        return len(x) > 0 and all(ord(ch) != 0 for ch in x)
    raise MatlabError(f"condition of {x!r}")


# ----------------------------------------------------------------------------------------------
# operators
# ----------------------------------------------------------------------------------------------

def _num(x):
    if isinstance(x, (float, bool)):
        return x
    if isinstance(x, str):
        return arr(x) if len(x) != 1 else float(ord(x))
    if isinstance(x, np.ndarray):
        return x
    if isinstance(x, (np.floating, np.integer, np.bool_, int)):
        return float(x)
    raise MatlabError(f"operand {x!r}")


def _elem(f):
    def g(a, b):
        if isinstance(a, float) and isinstance(b, float):
            return f(a, b)
        a, b = _num(a), _num(b)
        if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
            return scal(np.asarray(f(np.asarray(a, dtype=float) if not isinstance(a, np.ndarray) else a.astype(float, copy=False),
                                     np.asarray(b, dtype=float) if not isinstance(b, np.ndarray) else b.astype(float, copy=False)),
                                   dtype=float))
        return float(f(float(a), float(b)))
    return g


def _div(a, b):
    try:
        return a / b
    except ZeroDivisionError:
        return float(np.float64(a) / np.float64(b))


def _pow(a, b):
    try:
        r = a ** b
    except ZeroDivisionError:
        return float(np.float64(a) ** np.float64(b))
    if isinstance(r, complex):
        return r
    return r


m_plus = _elem(lambda a, b: a + b)
m_minus = _elem(lambda a, b: a - b)
m_times = _elem(lambda a, b: a * b)
_rdiv_elem = _elem(_div)


def m_rdiv(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return _div(a, b)
    a, b = _num(a), _num(b)
    with np.errstate(divide="ignore", invalid="ignore"):
        return scal(np.asarray(a, dtype=float) / np.asarray(b, dtype=float)) if (
            isinstance(a, np.ndarray) or isinstance(b, np.ndarray)) else _div(float(a), float(b))


def m_pow(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return _pow(a, b)
    a, b = _num(a), _num(b)
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return scal(np.power(np.asarray(a, dtype=float), np.asarray(b, dtype=float)))
    return _pow(float(a), float(b))


def m_mtimes(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return a * b
    a, b = _num(a), _num(b)
    if not isinstance(a, np.ndarray) or not isinstance(b, np.ndarray) or a.size == 1 or b.size == 1:
        return m_times(a, b)
    if a.shape[1] != b.shape[0]:
        raise MatlabError(f"mtimes: {a.shape} * {b.shape}")
    return scal(a.astype(float) @ b.astype(float))


def m_mrdiv(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return _div(a, b)
    b2 = _num(b)
    if isinstance(b2, np.ndarray) and b2.size != 1:
        raise MatlabError("matrix right division not supported")
    return m_rdiv(a, b)


def m_mpow(a, b):
    if isinstance(a, float) and isinstance(b, float):
        return _pow(a, b)
    a, b = _num(a), _num(b)
    if isinstance(a, np.ndarray) and a.size != 1:
        if not (isinstance(b, float) and b == int(b)):
            raise MatlabError("mpower: non-integer power of a matrix")
        if a.shape[0] != a.shape[1]:
            raise MatlabError("mpower: matrix must be square")
        if b < 0:
            a = np.linalg.inv(a)  # LAPACK getrf/getri family, as MATLAB's inv
            b = -b
        return np.linalg.matrix_power(a, int(b))
    return m_pow(a, b)


def m_neg(a):
    if isinstance(a, float):
        return -a
    a = _num(a)
    return -a if not isinstance(a, bool) else -float(a)


def m_not(a):
    if isinstance(a, (bool, float)):
        return not a
    a = _num(a)
    if isinstance(a, np.ndarray):
        return scal(a == 0)
    return a == 0


def _text_cmp(a, b):
    """== / ~= involving a string array (MATLAB compares whole texts)"""
    if isinstance(a, MStr) or isinstance(b, MStr):
        ta, tb = text_of(a), text_of(b)
        if ta is None or tb is None:
            return False
        return ta == tb
    return None


def _cmp(f):
    def g(a, b):
        if isinstance(a, float) and isinstance(b, float):
            return f(a, b)
        t = _text_cmp(a, b) if (isinstance(a, MStr) or isinstance(b, MStr)) else None
        if t is not None:
            return t if f(0.0, 0.0) else (not t)
        a, b = _num(a), _num(b)
        if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
            return scal(np.asarray(f(np.asarray(a, dtype=float), np.asarray(b, dtype=float))))
        return bool(f(float(a), float(b)))
    return g


m_eq = _cmp(lambda a, b: a == b)
m_ne = _cmp(lambda a, b: a != b)
m_lt = _cmp(lambda a, b: a < b)
m_le = _cmp(lambda a, b: a <= b)
m_gt = _cmp(lambda a, b: a > b)
m_ge = _cmp(lambda a, b: a >= b)


def m_and(a, b):
    a, b = _num(a), _num(b)
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return scal(np.logical_and(a, b))
    return bool(a) and bool(b)


def m_or(a, b):
    a, b = _num(a), _num(b)
    if isinstance(a, np.ndarray) or isinstance(b, np.ndarray):
        return scal(np.logical_or(a, b))
    return bool(a) or bool(b)


def m_transpose(a):
    if isinstance(a, (float, bool)):
        return a
    if isinstance(a, np.ndarray):
        return a.T.copy()
    if isinstance(a, MCell):
        return MCell(a.a.T.copy())
    if isinstance(a, MStr):
        return MStr(a.a.T.copy())
    if isinstance(a, str):
        if len(a) <= 1:
            return a
        raise MatlabError("char column vectors not supported")
    raise MatlabError(f"transpose of {a!r}")


def m_range(a, s, b):
    a = float(scal(_num(a)))
    b = float(scal(_num(b)))
    s = 1.0 if s is None else float(scal(_num(s)))
    if s == 0 or (s > 0 and a > b) or (s < 0 and a < b):
        return np.zeros((1, 0))
    n = int(math.floor((b - a) / s * (1 + 1e-15) + 1e-10)) + 1
    return (a + s * np.arange(n, dtype=float)).reshape(1, n)


def m_frange(a, s, b):
    r = m_range(a, s, b)
    return [float(v) for v in r[0]]


def m_for(x):
    if isinstance(x, (float, bool)):
        return [x]
    if isinstance(x, np.ndarray):
        if x.shape[0] == 1:
            return [scal(v) for v in x[0]]
        return [x[:, j:j + 1].copy() for j in range(x.shape[1])]
    if isinstance(x, MCell):
        return [MCell(x.a[:, j:j + 1].copy()) for j in range(x.a.shape[1])]
    raise MatlabError(f"for over {x!r}")


# ----------------------------------------------------------------------------------------------
# indexing
# ----------------------------------------------------------------------------------------------

def m_end(obj, k, n):
    sh = shape_of(obj)
    if n == 1:
        return float(sh[0] * sh[1])
    if k == 0:
        return float(sh[0])
    return float(sh[1])


def _idx(s, extent):
    """subscript -> 0-based int array (or slice marker)"""
    if s is COLON:
        return np.arange(extent)
    if isinstance(s, (float, int, np.floating, np.integer)):
        v = float(s)
        if v != int(v) or v < 1:
            raise MatlabError(f"bad index {v}")
        return np.array([int(v) - 1])
    if isinstance(s, bool):
        return np.array([0]) if s else np.zeros(0, dtype=int)
    if isinstance(s, np.ndarray):
        if s.dtype == bool:
            return np.nonzero(s.reshape(-1, order="F"))[0]
        f = s.reshape(-1, order="F")
        if f.size and (np.any(f < 1) or np.any(f != np.floor(f))):
            raise MatlabError("bad index")
        return f.astype(np.int64) - 1
    raise MatlabError(f"index {s!r}")


def _is_scalar_sub(s):
    return isinstance(s, (float, int, np.floating, np.integer)) and not isinstance(s, bool)


def _lin_shape(src_shape, s, n):
    """result shape of linear indexing src(s)"""
    if s is COLON:
        return (n, 1)
    ishape = shape_of(s) if not isinstance(s, (float, int)) else (1, 1)
    if src_shape[0] == 1 and len(ishape) == 2 and (ishape[0] == 1 or ishape[1] == 1):
        return (1, n)
    if src_shape[1] == 1 and src_shape[0] != 1 and (ishape[0] == 1 or ishape[1] == 1):
        return (n, 1)
    return ishape


def _grid(a, subs):
    """values array a (2-D, any dtype) -> selected sub-array"""
    if len(subs) == 1:
        s = subs[0]
        flat = a.reshape(-1, order="F")
        ii = _idx(s, flat.size)
        if ii.size and ii.max() >= flat.size:
            raise MatlabError("Index exceeds the number of array elements")
        out = flat[ii]
        return out.reshape(_lin_shape(a.shape, s, ii.size), order="F")
    if len(subs) == 2:
        r = _idx(subs[0], a.shape[0])
        c = _idx(subs[1], a.shape[1])
        if (r.size and r.max() >= a.shape[0]) or (c.size and c.max() >= a.shape[1]):
            raise MatlabError(f"Index exceeds matrix dimensions {a.shape}")
        return a[np.ix_(r, c)]
    raise MatlabError("more than 2 subscripts")


def m_paren(base, subs):
    if isinstance(base, np.ndarray):
        if len(subs) == 2 and _is_scalar_sub(subs[0]) and _is_scalar_sub(subs[1]):
            v = base[int(subs[0]) - 1, int(subs[1]) - 1]
            return bool(v) if base.dtype == bool else float(v)
        if len(subs) == 1 and _is_scalar_sub(subs[0]):
            k = int(subs[0]) - 1
            r = base.shape[0]
            if k < 0 or k >= base.size:
                raise MatlabError("Index exceeds the number of array elements")
            v = base[k % r, k // r]
            return bool(v) if base.dtype == bool else float(v)
        return scal(_grid(base, subs))
    if isinstance(base, (float, bool)):
        return scal(_grid(arr(base), subs))
    if isinstance(base, str):
        chars = np.array([[ch for ch in base]], dtype=object) if base else np.empty((0, 0), dtype=object)
        g = _grid(chars, subs)
        return "".join(g.reshape(-1, order="F"))
    if isinstance(base, MCell):
        return MCell(_grid(base.a, subs))
    if isinstance(base, MStr):
        return MStr(_grid(base.a, subs))
    if isinstance(base, MStruct):
        ids = np.arange(len(base.elems)).reshape(1, -1)
        g = _grid(ids, subs)
        return MStruct([base.elems[int(k)] for k in g.reshape(-1, order="F")], base.fields)
    raise MatlabError(f"index into {base!r}")


def m_brace(base, subs):
    if isinstance(base, MCell):
        if len(subs) == 2 and _is_scalar_sub(subs[0]) and _is_scalar_sub(subs[1]):
            return base.a[int(subs[0]) - 1, int(subs[1]) - 1]
        g = _grid(base.a, subs)
        vals = list(g.reshape(-1, order="F"))
        return vals[0] if len(vals) == 1 else CSList(vals)
    if isinstance(base, MStr):
        g = _grid(base.a, subs)
        vals = [v for v in g.reshape(-1, order="F")]
        return vals[0] if len(vals) == 1 else CSList(vals)
    raise MatlabError(f"brace index into {base!r}")


def m_field(base, name):
    if isinstance(base, MStruct):
        if len(base.elems) == 1:
            return base.get(0, name)
        return CSList([base.get(k, name) for k in range(len(base.elems))])
    raise MatlabError(f"field {name} of {base!r}")


def _default_for(val):
    if isinstance(val, MCell):
        return MCell.empty(0, 0)
    if isinstance(val, MStr):
        return MStr(np.empty((0, 0), dtype=object))
    if isinstance(val, str):
        return ""
    return np.zeros((0, 0))


def _grow(a, rows, cols, fill):
    if a.shape[0] >= rows and a.shape[1] >= cols:
        return a
    r, c = max(a.shape[0], rows), max(a.shape[1], cols)
    if a.dtype == object:
        b = np.empty((r, c), dtype=object)
        for idx in np.ndindex(r, c):
            b[idx] = fill() if callable(fill) else fill
    else:
        b = np.zeros((r, c), dtype=a.dtype)
    b[:a.shape[0], :a.shape[1]] = a
    return b


def _setgrid(a, subs, vals, fill):
    """a[subs] = vals (vals: 2-D array of the same kind, or 1x1 to broadcast); returns the array"""
    if len(subs) == 1:
        s = subs[0]
        n = a.size
        ii = _idx(s, n)
        need = int(ii.max()) + 1 if ii.size else 0
        if need > n:
            if a.shape[0] <= 1:
                a = _grow(a, 1, need, fill)
            elif a.shape[1] == 1:
                a = _grow(a, need, 1, fill)
            else:
                raise MatlabError("linear index growth of a matrix")
        r = a.shape[0]
        v = vals.reshape(-1, order="F")
        if v.size == 1:
            v = np.repeat(v, ii.size) if a.dtype != object else np.array([v[0]] * ii.size, dtype=object)
        if v.size != ii.size:
            raise MatlabError("In an assignment A(I) = B, the number of elements in B and I must be the same")
        for t, k in enumerate(ii):
            a[k % r, k // r] = v[t]
        return a
    r = _idx(subs[0], a.shape[0])
    c = _idx(subs[1], a.shape[1])
    a = _grow(a, int(r.max()) + 1 if r.size else 0, int(c.max()) + 1 if c.size else 0, fill)
    if vals.size == 1:
        a[np.ix_(r, c)] = vals.reshape(-1)[0]
        return a
    if vals.shape != (r.size, c.size):
        if vals.size != r.size * c.size:
            raise MatlabError(f"Subscripted assignment dimension mismatch {vals.shape} -> {(r.size, c.size)}")
        vals = vals.reshape((r.size, c.size), order="F")
    a[np.ix_(r, c)] = vals
    return a


def m_setparen(base, subs, val):
    if base is UNDEF:
        base = _default_for(val)
    if isinstance(base, MCell):
        if not isinstance(val, MCell):
            if isinstance(val, np.ndarray) and val.size == 0:
                raise MatlabError("deleting cell elements not supported")
            raise MatlabError("Conversion to cell from non-cell")
        base.a = _setgrid(base.a, subs, val.a, EMPTY)
        return base
    if isinstance(base, MStr):
        v = val.a if isinstance(val, MStr) else np.array([[text_of(val)]], dtype=object)
        base.a = _setgrid(base.a, subs, v, None)
        return base
    if isinstance(base, str):
        raise MatlabError("char assignment not supported")
    if isinstance(base, MStruct):
        raise MatlabError("struct paren assignment not supported")
    a = arr(base)
    v = arr(_num(val))
    if v.dtype == bool and a.dtype != bool:
        v = v.astype(float)
    if a.dtype == bool and v.dtype != bool:
        a = a.astype(float)
    if a is base:
        a = a  # in place
    elif isinstance(base, np.ndarray):
        pass
    if not a.flags.writeable:
        a = a.copy()
    return _setgrid(a, subs, v, 0.0)


def _struct_elem(base, subs):
    """base(subs) of a struct array for an assignment through it (grows); returns (base, k)"""
    if base is UNDEF or (isinstance(base, np.ndarray) and base.size == 0):
        base = MStruct([])
    if not isinstance(base, MStruct):
        raise MatlabError("struct element assignment on non-struct")
    if len(subs) == 2:
        if float(subs[0]) != 1:
            raise MatlabError("struct arrays are 1 x n here")
        s = subs[1]
    else:
        s = subs[0]
    k = int(float(s)) - 1
    while len(base.elems) <= k:
        base.elems.append({})
    return base, k


def m_assign(base, ops, val):
    """base<ops> = val; returns the new base (mutated in place where possible)"""
    if not ops:
        return val
    op, arg = ops[0]
    rest = ops[1:]
    if op == "f":
        if base is UNDEF or (isinstance(base, np.ndarray) and base.size == 0):
            base = MStruct()
        if not isinstance(base, MStruct) or len(base.elems) != 1:
            raise MatlabError(f"field assignment .{arg} on {base!r}")
        cur = base.elems[0].get(arg, UNDEF)
        base.elems[0][arg] = m_assign(cur, rest, val)
        if arg not in base.fields:
            base.fields.append(arg)
        return base
    if op == "p":
        if rest:
            base, k = _struct_elem(base, arg)
            elem = MStruct([base.elems[k]], base.fields)
            m_assign(elem, rest, val)
            for f in elem.fields:
                if f not in base.fields:
                    base.fields.append(f)
            return base
        return m_setparen(base, arg, val)
    if op == "b":
        if base is UNDEF:
            base = MCell.empty(0, 0)
        if not isinstance(base, MCell):
            raise MatlabError("brace assignment on non-cell")
        if rest:
            cur = m_brace(base, arg)
            new = m_assign(cur, rest, val)
        else:
            new = val
        holder = np.empty((1, 1), dtype=object)
        holder[0, 0] = new
        base.a = _setgrid(base.a, arg, holder, EMPTY)
        return base
    raise MatlabError(op)


# ----------------------------------------------------------------------------------------------
# concatenation
# ----------------------------------------------------------------------------------------------

def _flat_elems(row):
    out = []
    for e in row:
        if isinstance(e, CSList):
            out.extend(e)
        else:
            out.append(e)
    return out


def _is_empty(x):
    return isinstance(x, np.ndarray) and x.size == 0 or (isinstance(x, str) and x == "") or (
        isinstance(x, MCell) and x.a.size == 0)


def _hcat(items):
    items = [x for x in items if not _is_empty(x)] or items[:1]
    if not items:
        return np.zeros((0, 0))
    if any(isinstance(x, MCell) for x in items):
        parts = [x.a if isinstance(x, MCell) else _wrap_obj(x) for x in items]
        return MCell(np.hstack(parts))
    if any(isinstance(x, MStr) for x in items):
        parts = [x.a if isinstance(x, MStr) else np.array([[text_of(x) if is_text(x) else str(x)]], dtype=object)
                 for x in items]
        return MStr(np.hstack(parts))
    if all(isinstance(x, str) for x in items):
        return "".join(items)
    if any(isinstance(x, str) for x in items):
        return "".join(x if isinstance(x, str) else chr(int(scal(x))) for x in items)
    if len(items) == 1:
        x = items[0]
        return x.copy() if isinstance(x, np.ndarray) else x
    if all(isinstance(x, float) for x in items):
        return np.array([items], dtype=float)
    parts = [arr(_num(x)) for x in items]
    if any(p.dtype != bool for p in parts):
        parts = [p.astype(float) for p in parts]
    return np.hstack(parts)


def _wrap_obj(x):
    a = np.empty((1, 1), dtype=object)
    a[0, 0] = x
    return a


def _vcat(items):
    items = [x for x in items if not _is_empty(x)] or items[:1]
    if len(items) == 1:
        x = items[0]
        return x.copy() if isinstance(x, np.ndarray) else x
    if any(isinstance(x, MCell) for x in items):
        return MCell(np.vstack([x.a if isinstance(x, MCell) else _wrap_obj(x) for x in items]))
    if any(isinstance(x, MStr) for x in items):
        return MStr(np.vstack([x.a if isinstance(x, MStr) else np.array([[text_of(x)]], dtype=object) for x in items]))
    if any(isinstance(x, str) for x in items):
        raise MatlabError("char matrices not supported")
    if all(isinstance(x, float) for x in items):
        return np.array(items, dtype=float).reshape(-1, 1)
    parts = [arr(_num(x)) for x in items]
    if any(p.dtype != bool for p in parts):
        parts = [p.astype(float) for p in parts]
    return scal(np.vstack(parts)) if sum(p.size for p in parts) == 1 else np.vstack(parts)


def m_cat(rows):
    rows = [r for r in (_flat_elems(r) for r in rows) if r]
    if not rows:
        return np.zeros((0, 0))
    return _vcat([_hcat(r) for r in rows])


def m_cellcat(rows):
    rows = [r for r in (_flat_elems(r) for r in rows) if r]
    if not rows:
        return MCell.empty(0, 0)
    out = []
    for r in rows:
        out.append(np.hstack([_wrap_obj(x) for x in r]))
    return MCell(np.vstack(out))


def m_args(items):
    out = []
    for e in items:
        if isinstance(e, CSList):
            out.extend(e)
        else:
            out.append(e)
    return out


# ----------------------------------------------------------------------------------------------
# built-in functions (MATLAB library restated; not reference code)
# ----------------------------------------------------------------------------------------------

def _texts(x):
    """object ndarray of texts (None for non-text / missing) and whether x was scalar"""
    if isinstance(x, str):
        return x, True
    if isinstance(x, MStr):
        if x.a.size == 1:
            return x.a.flat[0], True
        return x.a, False
    if isinstance(x, MCell):
        a = np.empty(x.a.shape, dtype=object)
        for idx in np.ndindex(x.a.shape):
            v = x.a[idx]
            a[idx] = v if isinstance(v, str) else (text_of(v) if isinstance(v, MStr) and v.a.size == 1 else None)
        if a.size == 1:
            return a.flat[0], True
        return a, False
    return None, True


def b_strcmp(a, b):
    ta, sa = _texts(a)
    tb, sb = _texts(b)
    if sa and sb:
        return ta is not None and tb is not None and ta == tb
    if sa:
        ta, tb = tb, ta
    out = np.zeros(ta.shape, dtype=bool)
    for idx in np.ndindex(ta.shape):
        out[idx] = ta[idx] is not None and tb is not None and ta[idx] == tb
    return out


def b_size(x, d=None, nargout=1):
    r, c = shape_of(x)
    if d is not None:
        d = int(float(d))
        return float(r if d == 1 else c if d == 2 else 1)
    if nargout >= 2:
        return float(r), float(c)
    return np.array([[float(r), float(c)]])


def b_length(x):
    r, c = shape_of(x)
    return 0.0 if r == 0 or c == 0 else float(max(r, c))


def _dims(args):
    if len(args) == 0:
        return 1, 1
    if len(args) == 1:
        a = args[0]
        if isinstance(a, np.ndarray) and a.size == 2:
            return int(a.flat[0]), int(a.flat[1])
        n = int(float(scal(a)))
        return n, n
    return int(float(scal(args[0]))), int(float(scal(args[1])))


def b_zeros(*args):
    r, c = _dims(args)
    if r == 1 and c == 1:
        return 0.0
    return np.zeros((max(r, 0), max(c, 0)))


def b_cell(*args):
    r, c = _dims(args)
    return MCell.empty(max(r, 0), max(c, 0))


def _str2double_one(t):
    if t is None:
        return float("nan")
    s = t.strip()
    if not re.fullmatch(r"[+-]?(\d+\.?\d*|\.\d+)([eEdD][+-]?\d+)?|[+-]?(Inf|inf|NaN|nan)", s):
        return float("nan")
    return float(s.replace("d", "e").replace("D", "e"))


def b_str2double(x):
    if isinstance(x, str):
        return _str2double_one(x)
    if isinstance(x, MStr):
        if x.a.size == 1:
            return _str2double_one(x.a.flat[0])
        return np.vectorize(_str2double_one, otypes=[float])(x.a)
    if isinstance(x, MCell):
        t, s = _texts(x)
        if s:
            return _str2double_one(t)
        return np.vectorize(_str2double_one, otypes=[float])(t)
    return float("nan")


def b_char(x):
    if isinstance(x, str):
        return x
    if isinstance(x, MStr) and x.a.size == 1:
        return x.a.flat[0]
    if isinstance(x, MCell) and x.a.size == 1 and isinstance(x.a.flat[0], str):
        return x.a.flat[0]
    if isinstance(x, float):
        return chr(int(x))
    raise MatlabError(f"char({x!r})")


def b_num2str(x, fmt=None):
    if isinstance(x, str):
        return x
    x = scal(x)
    if isinstance(x, bool):
        x = float(x)
    if isinstance(x, float):
        if fmt is not None:
            return "%.*g" % (int(float(fmt)), x)
        if x == int(x) and abs(x) < 1e15:
            return str(int(x))
        return "%.5g" % x if abs(x) < 1e5 else "%.4g" % x
    return str(x)


def b_strcat(*args):
    if any(isinstance(a, MCell) for a in args):
        t = "".join(text_of(a.a.flat[0]) if isinstance(a, MCell) else text_of(a) for a in args)
        return MCell(_wrap_obj(t))
    if any(isinstance(a, MStr) for a in args):
        return MStr.scalar("".join(text_of(a) for a in args))
    return "".join(a.rstrip(" \t\n") for a in args)


def b_unique(x):
    if isinstance(x, MCell):
        t, _ = _texts(x)
        vals = sorted(set(v for v in np.asarray(t, dtype=object).reshape(-1)))
        a = np.empty((len(vals), 1), dtype=object)
        for i, v in enumerate(vals):
            a[i, 0] = v
        if x.a.shape[0] == 1:
            a = a.T.copy()
        return MCell(a)
    if isinstance(x, MStr):
        vals = sorted(set(v for v in x.a.reshape(-1) if v is not None))
        a = np.array(vals, dtype=object).reshape(-1, 1)
        return MStr(a.T.copy() if x.a.shape[0] == 1 else a)
    a = arr(_num(x))
    u = np.unique(a.reshape(-1))
    return scal(u.reshape(1, -1) if a.shape[0] == 1 else u.reshape(-1, 1))


def b_diag(v):
    a = arr(_num(v))
    if a.shape[0] == 1 or a.shape[1] == 1:
        return np.diag(a.reshape(-1))
    return np.diag(a).reshape(-1, 1).copy()


def b_repmat(a, m, n=None):
    if n is None:
        m, n = _dims([m])
    a = arr(_num(a))
    return np.tile(a, (int(float(m)), int(float(n))))


def _math1(fn_scalar, fn_arr):
    def g(x):
        if isinstance(x, float):
            try:
                return fn_scalar(x)
            except (ValueError, OverflowError):
                return complex(fn_arr(np.complex128(x)))
        x = _num(x)
        if isinstance(x, np.ndarray):
            return scal(fn_arr(x.astype(float)))
        return g(float(x))
    return g


b_sqrt = _math1(math.sqrt, np.sqrt)
b_sin = _math1(math.sin, np.sin)
b_cos = _math1(math.cos, np.cos)
b_tan = _math1(math.tan, np.tan)
b_atan = _math1(math.atan, np.arctan)
b_sec = _math1(lambda v: 1.0 / math.cos(v), lambda v: 1.0 / np.cos(v))
b_abs = _math1(abs, np.abs)


def b_atan2(y, x):
    if isinstance(y, float) and isinstance(x, float):
        return math.atan2(y, x)
    return scal(np.arctan2(arr(_num(y)), arr(_num(x))))


def b_sum(x):
    if isinstance(x, (float, bool)):
        return float(x)
    a = arr(_num(x)).astype(float)
    if a.shape[0] == 1:
        return float(np.sum(a)) if a.size else 0.0  # MATLAB sums a row vector along it
    if a.size == 0:
        return 0.0
    # column sums, in index order (MATLAB's summation order for a column)
    out = np.zeros((1, a.shape[1]))
    for j in range(a.shape[1]):
        s = 0.0
        for v in a[:, j]:
            s += float(v)
        out[0, j] = s
    return scal(out)


def b_mean(x):
    a = arr(_num(x)).astype(float)
    if a.shape[0] == 1:
        return b_sum(a) / a.shape[1]
    return scal(arr(b_sum(a)) / a.shape[0])


def b_isnan(x):
    if isinstance(x, float):
        return math.isnan(x)
    if isinstance(x, str):
        return scal(np.zeros((1, len(x)), dtype=bool)) if x else np.zeros((0, 0), dtype=bool)
    return scal(np.isnan(arr(_num(x))))


def b_ismissing(x):
    if isinstance(x, MStr):
        return scal(np.vectorize(lambda v: v is None, otypes=[bool])(x.a))
    if isinstance(x, float):
        return math.isnan(x)
    return False


def b_isempty(x):
    r, c = shape_of(x)
    return r == 0 or c == 0


def b_rmfield(s, name):
    name = text_of(name)
    if not isinstance(s, MStruct) or name not in s.fields:
        raise MatlabError(f"rmfield: field '{name}' does not exist")
    out = copy.deepcopy(s)
    out.fields.remove(name)
    for e in out.elems:
        e.pop(name, None)
    return out


def b_fileparts(p, nargout=1):
    p = text_of(p)
    d, f = os.path.split(p)
    name, ext = os.path.splitext(f)
    out = (d, name, ext)
    return out[:nargout] if nargout > 1 else out[0]


def _cwd_builtins(interp):
    def b_pwd():
        return interp.cwd

    def b_cd(d):
        interp.cwd = os.path.join(interp.cwd, text_of(d))
        return None

    def b_dir(pattern):
        pattern = text_of(pattern)
        base = os.path.join(interp.cwd, os.path.dirname(pattern))
        pat = os.path.basename(pattern)
        names = sorted(f for f in os.listdir(base) if fnmatch.fnmatchcase(f, pat))
        elems = [{"name": n, "folder": base, "isdir": os.path.isdir(os.path.join(base, n))} for n in names]
        return MStruct(elems, ["name", "folder", "isdir"])

    def b_readmatrix(path, *opts):
        """readmatrix(path, 'FileType','text', 'NumHeaderLines',0, 'Delimiter',{' ','\\t'},
        'ConsecutiveDelimitersRule','join', 'LeadingDelimitersRule','ignore', 'OutputType','string',
        'CommentStyle','#') -- the option set ReadFiles.m passes (ReadFiles.m:49), and only it: text
        after '#' dropped, runs of blanks / tabs one delimiter, leading ones ignored, empty lines
        skipped (the default EmptyLineRule), the result a string array as wide as the widest row,
        shorter rows padded with <missing>."""
        o = {text_of(opts[i]): opts[i + 1] for i in range(0, len(opts), 2)}
        assert text_of(o["OutputType"]) == "string" and text_of(o["CommentStyle"]) == "#"
        assert text_of(o["ConsecutiveDelimitersRule"]) == "join" and float(o["NumHeaderLines"]) == 0
        rows = []
        with open(os.path.join(interp.cwd, text_of(path))) as fh:
            for line in fh:
                line = line.split("#", 1)[0]
                toks = line.replace("\t", " ").split()
                if toks:
                    rows.append(toks)
        w = max((len(r) for r in rows), default=0)
        a = np.empty((len(rows), w), dtype=object)
        for i, r in enumerate(rows):
            for j in range(w):
                a[i, j] = r[j] if j < len(r) else None
        return MStr(a)

    return {"pwd": b_pwd, "cd": b_cd, "dir": b_dir, "readmatrix": b_readmatrix}


def _gui(name):
    def g(*a, **k):
        raise MatlabError(f"{name}() reached: the run took a GUI branch")
    return g


BUILTINS = {
    "size": b_size, "length": b_length, "zeros": b_zeros, "cell": b_cell, "str2double": b_str2double,
    "char": b_char, "num2str": b_num2str, "strcat": b_strcat, "strcmp": b_strcmp, "unique": b_unique,
    "diag": b_diag, "repmat": b_repmat, "sqrt": b_sqrt, "sin": b_sin, "cos": b_cos, "tan": b_tan,
    "atan": b_atan, "atan2": b_atan2, "sec": b_sec, "abs": b_abs, "sum": b_sum, "mean": b_mean,
    "isnan": b_isnan, "ismissing": b_ismissing, "isempty": b_isempty, "rmfield": b_rmfield,
    "fileparts": b_fileparts, "pi": lambda: math.pi, "true": lambda: True, "false": lambda: False,
    "tic": lambda: None, "toc": lambda: 0.0,
    "errordlg": _gui("errordlg"), "questdlg": _gui("questdlg"), "uigetfile": _gui("uigetfile"),
    "waitfor": _gui("waitfor"), "uiwait": _gui("uiwait"),
}
NARGOUT_BUILTINS = {"size", "fileparts"}


# ----------------------------------------------------------------------------------------------
# tokenizer
# ----------------------------------------------------------------------------------------------

KEYWORDS = {"if", "elseif", "else", "end", "for", "while", "break", "continue", "return", "function",
            "switch", "case", "otherwise", "try", "catch"}
COMMANDS = {"clear", "close", "format", "hold", "clc", "figure"}
OPS = [".*", "./", ".^", ".'", ".\\", "==", "~=", "<=", ">=", "&&", "||",
       "+", "-", "*", "/", "\\", "^", "<", ">", "&", "|", "~", "!", "=", "(", ")", "[", "]", "{", "}",
       ",", ";", ":", ".", "@"]
NUM_RE = re.compile(r"(\d+\.?\d*|\.\d+)([eE][+-]?\d+)?")
ID_RE = re.compile(r"[A-Za-z_][A-Za-z0-9_]*")


class Tok:
    __slots__ = ("kind", "val", "line", "ws")

    def __init__(self, kind, val, line, ws):
        self.kind, self.val, self.line, self.ws = kind, val, line, ws

    def __repr__(self):
        return f"{self.kind}:{self.val!r}@{self.line}"


def _value_end(t):
    return t is not None and (t.kind in ("num", "str", "dstr", "id") or (t.kind == "kw" and t.val == "end")
                              or (t.kind == "op" and t.val in (")", "]", "}", "'", ".'")))


def tokenize(src):
    toks = []
    i, n, line = 0, len(src), 1
    stack = []  # '(' '[' '{' (literal) '{i' (index)
    ws = False
    stmt_start = True

    def prev():
        return toks[-1] if toks else None

    while i < n:
        ch = src[i]
        if ch == "\n":
            if stack and stack[-1] in ("[", "{"):
                toks.append(Tok("op", ";", line, ws))
            elif not stack:
                toks.append(Tok("nl", "\n", line, ws))
                stmt_start = True
            line += 1
            i += 1
            ws = False
            continue
        if ch in " \t\r":
            j = i
            while j < n and src[j] in " \t\r":
                j += 1
            if stack and stack[-1] in ("[", "{") and _value_end(prev()) and j < n:
                c2 = src[j]
                c3 = src[j + 1] if j + 1 < n else ""
                starts = (c2.isalnum() or c2 in "_([{'\"@" or (c2 == "." and c3.isdigit())
                          or (c2 == "~" and c3 != "=")
                          or (c2 in "+-" and c3 not in " \t=" and c3 != ""))
                if starts:
                    toks.append(Tok("op", ",", line, True))
            i = j
            ws = True
            continue
        if ch == "%":
            while i < n and src[i] != "\n":
                i += 1
            continue
        if stmt_start and not stack:
            m = ID_RE.match(src, i)
            if m and m.group(0) in COMMANDS:
                rest = src[m.end():]
                mm = re.match(r"[ \t]+([A-Za-z][^;\n%,]*)", rest)
                if mm or re.match(r"[ \t]*(;|\n|%|,|$)", rest):
                    arg = mm.group(1).strip() if mm else ""
                    toks.append(Tok("cmd", (m.group(0), arg), line, ws))
                    i = m.end() + (mm.end() if mm else 0)
                    stmt_start = False
                    ws = False
                    continue
        stmt_start = False
        if ch == "'":
            if _value_end(prev()) and not ws:
                toks.append(Tok("op", "'", line, ws))
                i += 1
                ws = False
                continue
            j = i + 1
            s = []
            while True:
                if j >= n or src[j] == "\n":
                    raise SyntaxError(f"unterminated string at line {line}")
                if src[j] == "'":
                    if j + 1 < n and src[j + 1] == "'":
                        s.append("'")
                        j += 2
                        continue
                    break
                s.append(src[j])
                j += 1
            toks.append(Tok("str", "".join(s), line, ws))
            i = j + 1
            ws = False
            continue
        if ch == '"':
            j = i + 1
            s = []
            while True:
                if j >= n or src[j] == "\n":
                    raise SyntaxError(f"unterminated string at line {line}")
                if src[j] == '"':
                    if j + 1 < n and src[j + 1] == '"':
                        s.append('"')
                        j += 2
                        continue
                    break
                s.append(src[j])
                j += 1
            toks.append(Tok("dstr", "".join(s), line, ws))
            i = j + 1
            ws = False
            continue
        m = NUM_RE.match(src, i)
        if m and (ch.isdigit() or (ch == "." and i + 1 < n and src[i + 1].isdigit())):
            txt = m.group(0)
            end = m.end()
            if txt.endswith(".") and end < n and src[end] in "*/^\\'":
                txt = txt[:-1]
                end -= 1
            toks.append(Tok("num", float(txt), line, ws))
            i = end
            ws = False
            continue
        m = ID_RE.match(src, i)
        if m:
            w = m.group(0)
            toks.append(Tok("kw" if w in KEYWORDS else "id", w, line, ws))
            i = m.end()
            ws = False
            continue
        for op in OPS:
            if src.startswith(op, i):
                if op == ".'" and not (_value_end(prev()) and not ws):
                    continue
                if op in ("(", "["):
                    stack.append(op)
                elif op == "{":
                    stack.append("{i" if (_value_end(prev()) and not ws) else "{")
                elif op in (")", "]", "}"):
                    if stack:
                        stack.pop()
                if op in (";", ",") and not stack:
                    stmt_start = True
                toks.append(Tok("op", op, line, ws))
                i += len(op)
                ws = False
                break
        else:
            raise SyntaxError(f"unexpected {ch!r} at line {line}")
    toks.append(Tok("eof", None, line, False))
    return toks


# ----------------------------------------------------------------------------------------------
# parser
# ----------------------------------------------------------------------------------------------

class Parser:
    def __init__(self, toks):
        self.t = toks
        self.i = 0
        self.in_index = 0

    def peek(self, k=0):
        return self.t[self.i + k]

    def next(self):
        t = self.t[self.i]
        self.i += 1
        return t

    def at(self, kind, val=None, k=0):
        t = self.peek(k)
        return t.kind == kind and (val is None or t.val == val)

    def expect(self, kind, val=None):
        t = self.next()
        if t.kind != kind or (val is not None and t.val != val):
            raise SyntaxError(f"expected {kind} {val!r}, got {t!r}")
        return t

    def skip_sep(self):
        while self.at("nl") or self.at("op", ";") or self.at("op", ","):
            self.next()

    # ---- file ----
    def parse_file(self):
        self.skip_sep()
        funcs = []
        if self.at("kw", "function"):
            while self.at("kw", "function"):
                funcs.append(self.function())
                self.skip_sep()
            self.expect("eof")
            return funcs
        body = self.block(("eof",))
        return [("function", "__script__", [], [], body, 1)]

    def function(self):
        line = self.expect("kw", "function").line
        outs = []
        if self.at("op", "["):
            self.next()
            while not self.at("op", "]"):
                if self.at("op", ","):
                    self.next()
                    continue
                outs.append(self.expect("id").val)
            self.next()
            self.expect("op", "=")
            name = self.expect("id").val
        else:
            first = self.expect("id").val
            if self.at("op", "="):
                self.next()
                outs = [first]
                name = self.expect("id").val
            else:
                name = first
        params = []
        if self.at("op", "("):
            self.next()
            while not self.at("op", ")"):
                if self.at("op", ","):
                    self.next()
                    continue
                t = self.next()
                params.append("~" if t.val in ("~", "!") else t.val)
            self.next()
        body = self.block(("end",))
        self.expect("kw", "end")
        return ("function", name, params, outs, body, line)

    def block(self, terms):
        out = []
        while True:
            self.skip_sep()
            t = self.peek()
            if t.kind == "eof" and "eof" in terms:
                return out
            if t.kind == "kw" and t.val in terms:
                return out
            if t.kind == "eof":
                raise SyntaxError("unexpected end of file")
            out.append(self.statement())

    def statement(self):
        t = self.peek()
        line = t.line
        if t.kind == "cmd":
            self.next()
            return ("cmd", t.val[0], t.val[1], line)
        if t.kind == "kw":
            if t.val == "if":
                self.next()
                clauses = [(self.expr(), self.block(("elseif", "else", "end")))]
                els = None
                while True:
                    k = self.next()
                    if k.val == "elseif":
                        clauses.append((self.expr(), self.block(("elseif", "else", "end"))))
                    elif k.val == "else":
                        els = self.block(("end",))
                    else:
                        break
                return ("if", clauses, els, line)
            if t.val == "for":
                self.next()
                paren = self.at("op", "(")
                if paren:
                    self.next()
                var = self.expect("id").val
                self.expect("op", "=")
                e = self.expr()
                if paren:
                    self.expect("op", ")")
                body = self.block(("end",))
                self.expect("kw", "end")
                return ("for", var, e, body, line)
            if t.val == "while":
                self.next()
                c = self.expr()
                body = self.block(("end",))
                self.expect("kw", "end")
                return ("while", c, body, line)
            if t.val in ("break", "continue", "return"):
                self.next()
                return (t.val, line)
            raise SyntaxError(f"unsupported keyword {t!r}")
        if t.kind == "op" and t.val == "[" and self._multi_assign():
            self.next()
            lhs = []
            while not self.at("op", "]"):
                if self.at("op", ","):
                    self.next()
                    continue
                if self.at("op", "~") or self.at("op", "!"):
                    self.next()
                    lhs.append(("tilde",))
                    continue
                lhs.append(self.postfix())
            self.next()
            self.expect("op", "=")
            return ("assign", lhs, self.expr(), line)
        e = self.expr()
        if self.at("op", "="):
            self.next()
            return ("assign", [e], self.expr(), line)
        return ("expr", e, line)

    def _multi_assign(self):
        depth, k = 0, self.i
        while True:
            t = self.t[k]
            if t.kind in ("eof", "nl"):
                return False
            if t.kind == "op" and t.val in ("(", "[", "{"):
                depth += 1
            elif t.kind == "op" and t.val in (")", "]", "}"):
                depth -= 1
                if depth == 0:
                    nt = self.t[k + 1]
                    return nt.kind == "op" and nt.val == "="
            k += 1

    # ---- expressions ----
    def expr(self):
        return self.oror()

    def _binloop(self, sub, ops):
        a = sub()
        while self.peek().kind == "op" and self.peek().val in ops:
            op = self.next().val
            a = ("bin", op, a, sub())
        return a

    def oror(self):
        return self._binloop(self.andand, ("||",))

    def andand(self):
        return self._binloop(self.orop, ("&&",))

    def orop(self):
        return self._binloop(self.andop, ("|",))

    def andop(self):
        return self._binloop(self.cmp, ("&",))

    def cmp(self):
        return self._binloop(self.rng, ("==", "~=", "<", "<=", ">", ">="))

    def rng(self):
        a = self.additive()
        if self.at("op", ":") and not self._colon_alone():
            self.next()
            b = self.additive()
            if self.at("op", ":") and not self._colon_alone():
                self.next()
                c = self.additive()
                return ("range", a, b, c)
            return ("range", a, None, b)
        return a

    def _colon_alone(self):
        nt = self.peek(1)
        return nt.kind == "op" and nt.val in (",", ")", "}")

    def additive(self):
        return self._binloop(self.mult, ("+", "-"))

    def mult(self):
        return self._binloop(self.unary, ("*", "/", ".*", "./", "\\", ".\\"))

    def unary(self):
        if self.peek().kind == "op" and self.peek().val in ("-", "+", "~", "!"):
            op = self.next().val
            return ("un", "~" if op == "!" else op, self.unary())
        return self.power()

    def power(self):
        a = self.postfix()
        while self.peek().kind == "op" and self.peek().val in ("^", ".^"):
            op = self.next().val
            a = ("bin", op, a, self.powarg())
        return a

    def powarg(self):
        if self.peek().kind == "op" and self.peek().val in ("-", "+", "~", "!"):
            op = self.next().val
            return ("un", "~" if op == "!" else op, self.powarg())
        return self.postfix()

    def args(self, close):
        out = []
        self.in_index += 1
        while not self.at("op", close):
            if self.at("op", ","):
                self.next()
                continue
            if self.at("op", ":") and self._colon_alone():
                self.next()
                out.append(("colon",))
                continue
            out.append(self.expr())
        self.next()
        self.in_index -= 1
        return out

    def postfix(self):
        a = self.primary()
        while True:
            t = self.peek()
            if t.kind != "op":
                return a
            if t.val == "(" and not (t.ws and self._in_literal()):
                self.next()
                a = ("call", a, self.args(")"))
            elif t.val == "{" and not t.ws:
                self.next()
                a = ("brace", a, self.args("}"))
            elif t.val == "." and self.peek(1).kind == "id" and not t.ws:
                self.next()
                a = ("field", a, self.next().val)
            elif t.val in ("'", ".'"):
                self.next()
                a = ("post", t.val, a)
            else:
                return a

    def _in_literal(self):
        return False

    def primary(self):
        t = self.next()
        if t.kind == "num":
            return ("num", t.val)
        if t.kind == "str":
            return ("str", t.val)
        if t.kind == "dstr":
            return ("dstr", t.val)
        if t.kind == "id":
            return ("id", t.val)
        if t.kind == "kw" and t.val == "end" and self.in_index > 0:
            return ("end",)
        if t.kind == "op":
            if t.val == "(":
                saved = self.in_index
                e = self.expr()
                self.expect("op", ")")
                self.in_index = saved
                return ("paren", e)
            if t.val == "[":
                return ("matrix", self.rows("]"))
            if t.val == "{":
                return ("cell", self.rows("}"))
            if t.val == "@":
                if self.at("op", "("):
                    self.next()
                    params = []
                    while not self.at("op", ")"):
                        tt = self.next()
                        if tt.kind == "id":
                            params.append(tt.val)
                    self.next()
                    return ("anon", params, self.expr())
                return ("fhandle", self.expect("id").val)
            if t.val == ":":
                return ("colon",)
        raise SyntaxError(f"unexpected token {t!r}")

    def rows(self, close):
        rows, cur = [], []
        while True:
            if self.at("op", close):
                self.next()
                if cur:
                    rows.append(cur)
                return rows
            if self.at("op", ";") or self.at("nl"):
                self.next()
                if cur:
                    rows.append(cur)
                cur = []
                continue
            if self.at("op", ","):
                self.next()
                continue
            cur.append(self.expr())


# ----------------------------------------------------------------------------------------------
# compiler (AST -> Python source)
# ----------------------------------------------------------------------------------------------

BINOPS = {"+": "m_plus", "-": "m_minus", "*": "m_mtimes", "/": "m_mrdiv", "^": "m_mpow", ".*": "m_times",
          "./": "m_rdiv", ".^": "m_pow", "==": "m_eq", "~=": "m_ne", "<": "m_lt", "<=": "m_le", ">": "m_gt",
          ">=": "m_ge", "&": "m_and", "|": "m_or"}
FAST_BIN = {"+": "+", "-": "-", "*": "*", "/": "/", ".*": "*", "./": "/", "^": "**", ".^": "**"}
FAST_FN = {"sin": "_ms.sin", "cos": "_ms.cos", "tan": "_ms.tan", "atan": "_ms.atan", "sqrt": "_ms.sqrt"}


def _assigned_names(body, acc):
    for st in body:
        k = st[0]
        if k == "assign":
            for lv in st[1]:
                b = lv
                while b[0] in ("call", "brace", "field"):
                    b = b[1]
                if b[0] == "id":
                    acc.add(b[1])
        elif k == "if":
            for _, bl in st[1]:
                _assigned_names(bl, acc)
            if st[2]:
                _assigned_names(st[2], acc)
        elif k == "for":
            acc.add(st[1])
            _assigned_names(st[3], acc)
        elif k == "while":
            _assigned_names(st[2], acc)
    return acc


class FuncCompiler:
    def __init__(self, name, params, outs, body, is_main=False):
        self.name, self.params, self.outs, self.body = name, params, outs, body
        self.vars = _assigned_names(body, set(p for p in params if p != "~") | set(outs))
        self.is_main = is_main
        self.tmp = 0
        self.lines = []
        self.endctx = []

    def newtmp(self):
        self.tmp += 1
        return f"_t{self.tmp}"

    def v(self, name):
        return "v_" + name

    # ---- expressions ----
    def ex(self, e):
        k = e[0]
        if k == "num":
            return repr(float(e[1]))
        if k == "str":
            return repr(e[1])
        if k == "dstr":
            return f"MStr.scalar({e[1]!r})"
        if k == "paren":
            return self.ex(e[1])
        if k == "id":
            nm = e[1]
            if nm in ("nargin", "nargout"):
                return "_" + nm
            if nm in self.vars:
                return self.v(nm)
            return f"_call({nm!r}, [], 1)"
        if k == "colon":
            return "COLON"
        if k == "end":
            if not self.endctx:
                raise SyntaxError("end outside an index")
            tmp, pos, n = self.endctx[-1]
            return f"m_end({tmp}, {pos}, {n})"
        if k == "range":
            return f"m_range({self.ex(e[1])}, {self.ex(e[2]) if e[2] is not None else 'None'}, {self.ex(e[3])})"
        if k == "bin":
            op = e[1]
            if op == "&&":
                return f"(m_true({self.ex(e[2])}) and m_true({self.ex(e[3])}))"
            if op == "||":
                return f"(m_true({self.ex(e[2])}) or m_true({self.ex(e[3])}))"
            return f"{BINOPS[op]}({self.ex(e[2])}, {self.ex(e[3])})"
        if k == "un":
            if e[1] == "-":
                return f"m_neg({self.ex(e[2])})"
            if e[1] == "+":
                return self.ex(e[2])
            return f"m_not({self.ex(e[2])})"
        if k == "post":
            return f"m_transpose({self.ex(e[2])})"
        if k == "call":
            base, args = e[1], e[2]
            if base[0] == "id" and base[1] not in self.vars and base[1] not in ("nargin", "nargout"):
                return f"_call({base[1]!r}, m_args([{', '.join(self.ex(a) for a in args)}]), 1)"
            return self.index_expr("m_paren", base, args)
        if k == "brace":
            return self.index_expr("m_brace", e[1], e[2])
        if k == "field":
            return f"m_field({self.ex(e[1])}, {e[2]!r})"
        if k == "matrix":
            return "m_cat([" + ", ".join("[" + ", ".join(self.ex(x) for x in r) + "]" for r in e[1]) + "])"
        if k == "cell":
            return "m_cellcat([" + ", ".join("[" + ", ".join(self.ex(x) for x in r) + "]" for r in e[1]) + "])"
        if k == "anon":
            return "None"
        if k == "fhandle":
            return f"FuncHandle({e[1]!r})"
        raise SyntaxError(f"cannot compile {k}")

    def index_expr(self, fn, base, args):
        tmp = self.newtmp()
        n = len(args)
        parts = []
        for pos, a in enumerate(args):
            self.endctx.append((tmp, pos, n))
            parts.append(self.ex(a))
            self.endctx.pop()
        return f"{fn}(({tmp} := {self.ex(base)}), m_args([{', '.join(parts)}]))"

    # ---- scalar fast path ----
    def fast(self, e, leaves):
        k = e[0]
        if k == "num":
            return repr(float(e[1]))
        if k == "paren":
            r = self.fast(e[1], leaves)
            return None if r is None else f"({r})"
        if k == "id":
            if e[1] in self.vars:
                leaves.add(e[1])
                return self.v(e[1])
            if e[1] == "pi":
                return repr(math.pi)
            return None
        if k == "bin" and e[1] in FAST_BIN:
            a = self.fast(e[2], leaves)
            b = self.fast(e[3], leaves)
            if a is None or b is None:
                return None
            return f"({a} {FAST_BIN[e[1]]} {b})"
        if k == "un" and e[1] in ("-", "+"):
            a = self.fast(e[2], leaves)
            return None if a is None else f"({e[1]}{a})"
        if k == "call" and e[1][0] == "id" and e[1][1] not in self.vars and len(e[2]) == 1:
            fn = e[1][1]
            a = self.fast(e[2][0], leaves)
            if a is None:
                return None
            if fn in FAST_FN:
                return f"{FAST_FN[fn]}({a})"
            if fn == "sec":
                return f"(1.0 / _ms.cos({a}))"
            if fn == "abs":
                return f"abs({a})"
        return None

    def size_of(self, e):
        return 1 + sum(self.size_of(x) for x in e[1:] if isinstance(x, tuple)) + sum(
            self.size_of(y) for x in e[1:] if isinstance(x, list) for y in x if isinstance(y, tuple))

    def rhs(self, e, ind):
        """emit code computing e into a temp; returns the temp name"""
        tmp = self.newtmp()
        leaves = set()
        fast = self.fast(e, leaves) if e[0] in ("bin", "un", "call", "paren") else None
        if fast is not None and leaves and self.size_of(e) >= 12:
            guard = " and ".join(f"isinstance({self.v(n)}, float)" for n in sorted(leaves))
            slow = self.ex(e)
            self.emit(ind, f"if {guard}:")
            self.emit(ind + 1, "try:")
            self.emit(ind + 2, f"{tmp} = {fast}")
            self.emit(ind + 1, "except (ZeroDivisionError, ValueError, OverflowError):")
            self.emit(ind + 2, f"{tmp} = {slow}")
            self.emit(ind, "else:")
            self.emit(ind + 1, f"{tmp} = {slow}")
            return tmp
        src = self.ex(e)
        if e[0] in ("id", "field") or (e[0] == "paren" and e[1][0] in ("id", "field")):
            src = f"m_cp({src})"
        self.emit(ind, f"{tmp} = {src}")
        return tmp

    # ---- statements ----
    def emit(self, ind, s):
        self.lines.append("    " * ind + s)

    def lvalue_ops(self, lv):
        ops = []
        b = lv
        while b[0] in ("call", "brace", "field"):
            if b[0] == "field":
                ops.append(f"('f', {b[2]!r})")
            else:
                for a in b[2]:
                    if self._has_end(a):
                        raise SyntaxError("end in an assignment subscript is not supported")
                args = ", ".join(self.ex(a) for a in b[2])
                ops.append(f"({'p' if b[0] == 'call' else 'b'!r}, m_args([{args}]))")
            b = b[1]
        if b[0] != "id":
            raise SyntaxError(f"bad lvalue {lv}")
        return b[1], list(reversed(ops))

    def _has_end(self, e):
        if not isinstance(e, tuple):
            return False
        if e[0] == "end":
            return True
        return any(self._has_end(x) for x in e[1:] if isinstance(x, tuple)) or any(
            self._has_end(y) for x in e[1:] if isinstance(x, list) for y in x)

    def assign_to(self, lv, src, ind):
        if lv[0] == "tilde":
            return
        name, ops = self.lvalue_ops(lv)
        self.vars.add(name)
        if not ops:
            self.emit(ind, f"{self.v(name)} = {src}")
        else:
            self.emit(ind, f"{self.v(name)} = m_assign({self.v(name)}, ({', '.join(ops)},), {src})")

    def stmts(self, body, ind):
        if not body:
            self.emit(ind, "pass")
        for st in body:
            self.stmt(st, ind)

    def stmt(self, st, ind):
        k = st[0]
        self.emit(ind, f"_line[0] = {st[-1]}" if k not in ("break", "continue", "return") else f"_line[0] = {st[1]}")
        if k == "assign":
            lhs, rhs = st[1], st[2]
            if len(lhs) == 1:
                tmp = self.rhs(rhs, ind)
                self.assign_to(lhs[0], tmp, ind)
                return
            if rhs[0] == "call" and rhs[1][0] == "id" and rhs[1][1] not in self.vars:
                args = ", ".join(self.ex(a) for a in rhs[2])
                call = f"_call({rhs[1][1]!r}, m_args([{args}]), {len(lhs)})"
            elif rhs[0] == "id" and rhs[1] not in self.vars:
                call = f"_call({rhs[1]!r}, [], {len(lhs)})"
            else:
                raise SyntaxError("multiple assignment from a non-call")
            tmp = self.newtmp()
            self.emit(ind, f"{tmp} = {call}")
            for q, lv in enumerate(lhs):
                self.assign_to(lv, f"{tmp}[{q}]", ind)
            return
        if k == "expr":
            e = st[1]
            if e[0] == "call" and e[1][0] == "id" and e[1][1] not in self.vars:
                args = ", ".join(self.ex(a) for a in e[2])
                self.emit(ind, f"_call({e[1][1]!r}, m_args([{args}]), 0)")
            elif e[0] == "id" and e[1] not in self.vars:
                self.emit(ind, f"_call({e[1]!r}, [], 0)")
            else:
                self.emit(ind, f"_ = {self.ex(e)}")
            return
        if k == "cmd":
            return
        if k == "if":
            for q, (c, bl) in enumerate(st[1]):
                self.emit(ind, f"{'if' if q == 0 else 'elif'} m_true({self.ex(c)}):")
                self.stmts(bl, ind + 1)
            if st[2] is not None:
                self.emit(ind, "else:")
                self.stmts(st[2], ind + 1)
            return
        if k == "for":
            self.vars.add(st[1])
            e = st[2]
            if e[0] == "range":
                it = f"m_frange({self.ex(e[1])}, {self.ex(e[2]) if e[2] is not None else 'None'}, {self.ex(e[3])})"
            else:
                it = f"m_for({self.ex(e)})"
            self.emit(ind, f"for {self.v(st[1])} in {it}:")
            self.stmts(st[3], ind + 1)
            return
        if k == "while":
            self.emit(ind, f"while m_true({self.ex(st[1])}):")
            self.stmts(st[2], ind + 1)
            return
        if k in ("break", "continue"):
            self.emit(ind, k)
            return
        if k == "return":
            if self.is_main:
                self.emit(ind, "raise MainReturn()")
            else:
                self.emit(ind, "return _outs(locals())")
            return
        raise SyntaxError(f"statement {k}")

    def compile(self):
        self.stmts(self.body, 1)
        body = self.lines
        self.lines = []
        self.emit(0, f"def f_{self.name}(*_a, nargout=1, _init=None):")
        self.emit(1, f"_line = _LINE[{self.name!r}]")
        self.emit(1, "_nargin = float(len(_a))")
        self.emit(1, "_nargout = float(nargout)")
        for q, p in enumerate(self.params):
            if p == "~":
                continue
            if p == "varargin":
                self.emit(1, f"v_varargin = MCell(np.array([list(_a[{q}:])], dtype=object)) "
                             f"if len(_a) > {q} else MCell.empty(1, 0)")
            else:
                self.emit(1, f"v_{p} = _a[{q}] if len(_a) > {q} else UNDEF")
        for n in sorted(self.vars):  # every other variable starts undefined
            if n not in self.params:
                self.emit(1, f"{self.v(n)} = UNDEF")
                if self.is_main:
                    self.emit(1, f"if {n!r} in _init: {self.v(n)} = _init[{n!r}]")
        outs = list(self.outs)
        self.emit(1, "def _outs(L):")
        if self.is_main:
            self.emit(2, "return {k[2:]: v for k, v in L.items() if k.startswith('v_')}")
        else:
            self.emit(2, f"o = [L.get(o, UNDEF) for o in {['v_' + o for o in outs]!r}]")
            self.emit(2, "return o[0] if nargout <= 1 and o else tuple(o[:max(nargout, 1)])")
        self.lines.extend(body)
        self.emit(1, "return _outs(locals())")
        return "\n".join(self.lines) + "\n"


# ----------------------------------------------------------------------------------------------
# interpreter
# ----------------------------------------------------------------------------------------------

class Interp:
    def __init__(self, verbose=False):
        self.funcs = {}
        self.user = {}
        self.cwd = os.getcwd()
        self.verbose = verbose
        self.hooks = {}  # name -> callback(args, outputs)
        self.builtins = dict(BUILTINS)
        self.builtins.update(_cwd_builtins(self))
        self.builtins["disp"] = self._disp
        self.lines = {}
        self.ns = {}
        for k, val in list(globals().items()):
            if k.startswith("m_") or k in ("MStr", "MCell", "MStruct", "UNDEF", "COLON", "np", "FuncHandle",
                                           "MainReturn", "CSList"):
                self.ns[k] = val
        self.ns["_ms"] = math
        self.ns["_call"] = self.call
        self.ns["_LINE"] = self.lines

    def _disp(self, x):
        if self.verbose:
            print(x if isinstance(x, str) else repr(x))

    def load_file(self, path, main_slice=None):
        """parse a .m file; its functions become callable.  main_slice=(name, first, last, init_names):
        instead of function `name` itself, compile the top-level statements of its body that start
        on lines first..last as `name`, run by run_slice with the variables init_names preset."""
        with open(path) as fh:
            src = fh.read()
        funcs = Parser(tokenize(src)).parse_file()
        for f in funcs:
            _, name, params, outs, body, _line = f
            if main_slice and name == main_slice[0]:
                first, last, init_names = main_slice[1], main_slice[2], main_slice[3]
                sel = [st for st in body if first <= self._stline(st) <= last]
                self._compile(name, [], [], sel, is_main=True, extra_vars=init_names)
            else:
                self._compile(name, params, outs, body)
        return [f[1] for f in funcs]

    @staticmethod
    def _stline(st):
        return st[-1] if st[0] not in ("break", "continue", "return") else st[1]

    def _compile(self, name, params, outs, body, is_main=False, extra_vars=()):
        fc = FuncCompiler(name, params, outs, body, is_main=is_main)
        fc.vars |= set(extra_vars)
        src = fc.compile()
        self.lines[name] = [0]
        code = compile(src, f"<mlang:{name}>", "exec")
        exec(code, self.ns)
        self.user[name] = self.ns["f_" + name]
        self.funcs[name] = (params, outs, body)

    def call(self, name, args, nargout):
        if name in self.user:
            args = [copy.deepcopy(a) if isinstance(a, (np.ndarray, MCell, MStruct, MStr)) else a for a in args]
            try:
                out = self.user[name](*args, nargout=nargout)
            except MatlabError as e:
                raise MatlabError(f"{e} (in {name} line {self.lines[name][0]})") from None
            if name in self.hooks:
                self.hooks[name](args, out)
            return out
        if name in self.builtins:
            f = self.builtins[name]
            if name in NARGOUT_BUILTINS:
                return f(*args, nargout=max(nargout, 1))
            return f(*args)
        raise MatlabError(f"Undefined function '{name}'")

    def run_slice(self, name, init):
        """run the compiled slice of `name` with the given initial variables; returns its variables"""
        f = self.user[name]
        try:
            return f(_init=init, nargout=0)
        except MainReturn:
            raise MatlabError(f"{name} returned early at line {self.lines[name][0]}") from None
        except MatlabError as e:
            raise MatlabError(f"{e} (in {name} line {self.lines[name][0]})") from None
