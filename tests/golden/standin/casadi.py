'''
Arithmetic-only stand-in for the part of the CasADi Python API that the reference's transcription
calls (SURVEY.md 8(c) "optional stronger pin"). TEST INFRASTRUCTURE ONLY: it exists so that
tests/golden/make_transcription_golden.py can execute the reference's OWN row-building code
(/root/reference/drone3d/{raceline,dynamics,centerlines,utils}) in this container and dump
g(w), dg/dw, f(w), grad f(w), bounds and w0 as fixtures. It is never imported by the product,
by the GPU tests or by bench.py, and never travels to the GPU box.

It contains no transcription logic: only
  * an expression DAG of scalars (symbols, + - * / pow, sin cos tan sqrt exp log, comparisons,
    if_else) with the value-preserving folds CasADi's SX makes (x+0, x*1, 0*x, numbers),
  * SX / MX / DM matrix containers with CasADi's shape rules (column vectors by default,
    column-major linear indexing, scalar broadcasting, numpy interoperation),
  * Function (inline substitution for symbolic arguments, evaluation for numeric ones),
    jacobian (forward symbolic differentiation), and the published definitions of
    pw_const / pw_lin (sum of jumps), cumsum, norm_2, dot, cross, bilin, inv,
  * collocation_points: Gauss-Legendre roots on [0, 1] (mpmath, rounded once to double),
  * integrator / nlpsol: inert placeholders (construction only; calling them raises).
CasADi itself (third party, not in /root/reference, not installable offline: SURVEY F8) is
therefore replaced by plain IEEE arithmetic on the expressions the reference builds.
'''
import numbers

import numpy as np

__version__ = '3.5.5+standin'


# ------------------------------------------------------------------------------ scalar DAG
class _N:
    __slots__ = ('op', 'a', 'b', 'c', 'id', 'name')
    _count = 0

    def __init__(self, op, a=None, b=None, c=None, name=None):
        _N._count += 1
        self.op, self.a, self.b, self.c, self.id, self.name = op, a, b, c, _N._count, name

    def __repr__(self):
        return self.name if self.op == 'sym' else f'<{self.op}#{self.id}>'


def _num(x):
    return not isinstance(x, _N)


def _add(a, b):
    if _num(a) and _num(b):
        return a + b
    if _num(a) and a == 0:
        return b
    if _num(b) and b == 0:
        return a
    return _N('add', a, b)


def _sub(a, b):
    if _num(a) and _num(b):
        return a - b
    if _num(b) and b == 0:
        return a
    if _num(a) and a == 0:
        return _neg(b)
    if a is b:
        return 0.0
    return _N('sub', a, b)


def _mul(a, b):
    if _num(a) and _num(b):
        return a * b
    if (_num(a) and a == 0) or (_num(b) and b == 0):
        return 0.0
    if _num(a) and a == 1:
        return b
    if _num(b) and b == 1:
        return a
    if _num(a) and a == -1:
        return _neg(b)
    if _num(b) and b == -1:
        return _neg(a)
    return _N('mul', a, b)


def _div(a, b):
    if _num(a) and _num(b):
        return a / b if b != 0 else (np.inf if a > 0 else -np.inf if a < 0 else np.nan)
    if _num(a) and a == 0:
        return 0.0
    if _num(b) and b == 1:
        return a
    return _N('div', a, b)


def _neg(a):
    if _num(a):
        return -a
    if a.op == 'neg':
        return a.a
    return _N('neg', a)


def _pow(a, b):
    if _num(a) and _num(b):
        return float(np.power(float(a), float(b)))
    if _num(b) and b == 1:
        return a
    if _num(b) and b == 0:
        return 1.0
    if _num(b) and b == 2:
        return _N('sq', a)
    return _N('pow', a, b)


def _unary(op, f):
    def build(a):
        return float(f(a)) if _num(a) else _N(op, a)
    return build


_sin = _unary('sin', np.sin)
_cos = _unary('cos', np.cos)
_tan = _unary('tan', np.tan)
_sqrt = _unary('sqrt', np.sqrt)
_exp = _unary('exp', np.exp)
_log = _unary('log', np.log)


def _cmp(op, f):
    def build(a, b):
        if _num(a) and _num(b):
            return 1.0 if f(a, b) else 0.0
        return _N(op, a, b)
    return build


_ge = _cmp('ge', lambda a, b: a >= b)
_gt = _cmp('gt', lambda a, b: a > b)
_le = _cmp('le', lambda a, b: a <= b)
_lt = _cmp('lt', lambda a, b: a < b)
_eq = _cmp('eq', lambda a, b: a == b)
_ne = _cmp('ne', lambda a, b: a != b)


def _ifelse(c, a, b):
    if _num(c):
        return a if c != 0 else b
    return _N('if_else', c, a, b)


_BUILD = {'add': _add, 'sub': _sub, 'mul': _mul, 'div': _div, 'neg': _neg, 'pow': _pow,
          'sq': lambda a: _mul(a, a) if _num(a) else _N('sq', a),
          'sin': _sin, 'cos': _cos, 'tan': _tan, 'sqrt': _sqrt, 'exp': _exp, 'log': _log,
          'ge': _ge, 'gt': _gt, 'le': _le, 'lt': _lt, 'eq': _eq, 'ne': _ne, 'if_else': _ifelse}


def _re(x):
    return np.real(x)


def _truth(x):
    return np.where(x, 1.0, 0.0) if isinstance(x, np.ndarray) else (1.0 if x else 0.0)


# numeric evaluation; values may be floats or numpy arrays (real or complex: complex-step Jacobians)
_EVAL = {'add': lambda a, b: a + b, 'sub': lambda a, b: a - b, 'mul': lambda a, b: a * b,
         'div': np.divide, 'neg': lambda a: -a, 'sq': lambda a: a * a,
         'pow': lambda a, b: np.power(a, b),
         'sin': np.sin, 'cos': np.cos, 'tan': np.tan, 'sqrt': np.sqrt, 'exp': np.exp, 'log': np.log,
         'ge': lambda a, b: _truth(_re(a) >= _re(b)), 'gt': lambda a, b: _truth(_re(a) > _re(b)),
         'le': lambda a, b: _truth(_re(a) <= _re(b)), 'lt': lambda a, b: _truth(_re(a) < _re(b)),
         'eq': lambda a, b: _truth(_re(a) == _re(b)), 'ne': lambda a, b: _truth(_re(a) != _re(b)),
         'if_else': lambda c, a, b: np.where(_re(c) != 0, a, b) if isinstance(c, np.ndarray) else (
             a if c != 0 else b)}


def _topo(roots):
    ''' post-order of every node reachable from roots (iterative; the DAGs are deep) '''
    order, seen = [], set()
    stack = [(r, False) for r in roots if isinstance(r, _N)]
    while stack:
        n, done = stack.pop()
        if done:
            order.append(n)
            continue
        if n.id in seen:
            continue
        seen.add(n.id)
        stack.append((n, True))
        for ch in (n.a, n.b, n.c):
            if isinstance(ch, _N) and ch.id not in seen:
                stack.append((ch, False))
    return order


def _children(n):
    return [ch for ch in (n.a, n.b, n.c) if ch is not None] if n.op != 'sym' else []


def evaluate(order, leaf):
    ''' values of every node in order (leaf: sym id -> value); returns id -> value '''
    val = {}
    for n in order:
        if n.op == 'sym':
            if n.id not in leaf:
                raise RuntimeError(f'free symbol {n.name} in a numeric evaluation')
            val[n.id] = leaf[n.id]
            continue
        args = [val[ch.id] if isinstance(ch, _N) else ch for ch in _children(n)]
        val[n.id] = _EVAL[n.op](*args)
    return val


def _substitute(order, leaf):
    ''' rebuild the nodes with symbols replaced (leaf: sym id -> entry), folding numbers '''
    val = {}
    for n in order:
        if n.op == 'sym':
            val[n.id] = leaf.get(n.id, n)
            continue
        args = [val[ch.id] if isinstance(ch, _N) else ch for ch in _children(n)]
        val[n.id] = _BUILD[n.op](*args)
    return val


def _derivative(entries, x):
    ''' d entries / d x (x a symbol node), forward symbolic mode '''
    order = _topo(entries)
    d = {}

    def D(e):
        return d[e.id] if isinstance(e, _N) else 0.0

    for n in order:
        op, a, b = n.op, n.a, n.b
        if op == 'sym':
            r = 1.0 if n is x else 0.0
        elif op == 'add':
            r = _add(D(a), D(b))
        elif op == 'sub':
            r = _sub(D(a), D(b))
        elif op == 'neg':
            r = _neg(D(a))
        elif op == 'mul':
            r = _add(_mul(D(a), b), _mul(a, D(b)))
        elif op == 'div':
            r = _div(_sub(D(a), _mul(_div(a, b), D(b))), b)
        elif op == 'sq':
            r = _mul(_mul(2.0, a), D(a))
        elif op == 'pow':
            r = _mul(_mul(b, _pow(a, _sub(b, 1.0))), D(a))
            if isinstance(b, _N):
                r = _add(r, _mul(_mul(_log(a), n), D(b)))
        elif op == 'sin':
            r = _mul(_cos(a), D(a))
        elif op == 'cos':
            r = _neg(_mul(_sin(a), D(a)))
        elif op == 'tan':
            r = _mul(_add(1.0, _mul(n, n)), D(a))
        elif op == 'sqrt':
            r = _div(D(a), _mul(2.0, n))
        elif op == 'exp':
            r = _mul(n, D(a))
        elif op == 'log':
            r = _div(D(a), a)
        elif op in ('ge', 'gt', 'le', 'lt', 'eq', 'ne'):
            r = 0.0
        elif op == 'if_else':
            r = _ifelse(a, D(b), D(n.c))
        else:
            raise NotImplementedError(op)
        d[n.id] = r
    return [D(e) for e in entries]


# ------------------------------------------------------------------------------ matrices
def _entry(x):
    if isinstance(x, _N):
        return x
    if isinstance(x, _Mat):
        if x.m.size != 1:
            raise ValueError(f'expected a scalar, got {x.shape}')
        return x.m[0, 0]
    return float(x)


def _to_mat(x):
    ''' CasADi's implicit conversion of an operand to a matrix '''
    if isinstance(x, _Mat):
        return x
    if isinstance(x, _N):
        return SX._wrap(np.array([[x]], dtype=object))
    if isinstance(x, (numbers.Number, np.number, np.bool_)):
        return DM._wrap(np.array([[float(x)]], dtype=object))
    if isinstance(x, (list, tuple)):
        if len(x) and all(isinstance(e, (list, tuple, np.ndarray)) and np.ndim(e) == 1 for e in x):
            return _to_mat(np.array(x, dtype=object))
        return vertcat(*x) if len(x) else DM._wrap(np.zeros((0, 1), dtype=object))
    if isinstance(x, np.ndarray):
        if x.dtype == object:
            flat = [_entry(e) for e in x.reshape(-1)]
            a = np.empty(len(flat), dtype=object)
            a[:] = flat
            a = a.reshape(x.shape)
        else:
            a = x.astype(float).astype(object)
        if a.ndim == 0:
            a = a.reshape(1, 1)
        elif a.ndim == 1:
            a = a.reshape(-1, 1)
        cls = DM if all(_num(e) for e in a.reshape(-1)) else SX
        return cls._wrap(a)
    raise TypeError(f'cannot convert {type(x)} to a matrix')


def _result_cls(*ms):
    if any(isinstance(m, MX) for m in ms):
        return MX
    if any(isinstance(m, SX) for m in ms):
        return SX
    return DM


def _elementwise(fn, *ops):
    ms = [_to_mat(o) for o in ops]
    shape = None
    for m in ms:
        if m.shape != (1, 1):
            if shape is not None and m.shape != shape:
                raise ValueError(f'dimension mismatch {[mm.shape for mm in ms]}')
            shape = m.shape
    shape = shape or (1, 1)
    out = np.empty(shape, dtype=object)
    for i in range(shape[0]):
        for j in range(shape[1]):
            out[i, j] = fn(*[m.m[0, 0] if m.shape == (1, 1) else m.m[i, j] for m in ms])
    return _result_cls(*ms)._wrap(out)


def _index(k, n):
    if isinstance(k, slice):
        return list(range(*k.indices(n)))
    if isinstance(k, (list, tuple, np.ndarray)):
        return [int(i) % n for i in k]
    k = int(k)
    if k < -n or k >= n:
        raise IndexError(k)
    return [k % n]


class _Mat:
    __array_ufunc__ = None        # numpy operands defer to the reflected operators below
    __hash__ = object.__hash__

    def __init__(self, *args):
        if len(args) == 0:
            self.m = np.zeros((0, 0), dtype=object)
        elif len(args) == 2 and isinstance(args[0], str):
            self.m = type(self).sym(args[0], args[1]).m
        elif len(args) == 2 and all(isinstance(a, (int, np.integer)) for a in args):
            self.m = np.zeros((int(args[0]), int(args[1])), dtype=object)
            self.m[:] = 0.0
        elif len(args) == 1:
            self.m = _to_mat(args[0]).m.copy()
        else:
            raise TypeError(args)

    @classmethod
    def _wrap(cls, a):
        obj = cls.__new__(cls)
        obj.m = a
        return obj

    @classmethod
    def sym(cls, name, *dims):
        if len(dims) == 0:
            r, c = 1, 1
        elif len(dims) == 1 and isinstance(dims[0], (tuple, list)):
            r, c = (int(dims[0][0]), int(dims[0][1]) if len(dims[0]) > 1 else 1)
        elif len(dims) == 1:
            r, c = int(dims[0]), 1
        else:
            r, c = int(dims[0]), int(dims[1])
        a = np.empty((r, c), dtype=object)
        for j in range(c):
            for i in range(r):
                a[i, j] = _N('sym', name=f'{name}_{j * r + i}')
        return cls._wrap(a)

    # shape
    @property
    def shape(self):
        return self.m.shape

    def size(self):
        return self.m.shape

    def size1(self):
        return self.m.shape[0]

    def size2(self):
        return self.m.shape[1]

    def numel(self):
        return self.m.size

    def is_scalar(self):
        return self.m.size == 1

    @property
    def T(self):
        return type(self)._wrap(self.m.T.copy())

    def entries(self):
        ''' column-major entries (CasADi's nonzero order of a dense matrix) '''
        return list(self.m.T.reshape(-1))

    # indexing
    def _lin(self):
        return self.m.T.reshape(-1)

    def __getitem__(self, key):
        if isinstance(key, tuple):
            rows = _index(key[0], self.shape[0])
            cols = _index(key[1], self.shape[1])
            return type(self)._wrap(self.m[np.ix_(rows, cols)].copy())
        idx = _index(key, self.m.size)
        lin = self._lin()
        vals = np.empty(len(idx), dtype=object)
        vals[:] = [lin[i] for i in idx]
        shape = (1, len(idx)) if (self.shape[0] == 1 and self.shape[1] != 1) else (len(idx), 1)
        return type(self)._wrap(vals.reshape(shape))

    def __setitem__(self, key, value):
        v = _to_mat(value)
        if isinstance(key, tuple):
            rows = _index(key[0], self.shape[0])
            cols = _index(key[1], self.shape[1])
            pos = [(i, j) for j in cols for i in rows]
        else:
            r = self.shape[0]
            pos = [(i % r, i // r) for i in _index(key, self.m.size)]
        vals = [v.m[0, 0]] * len(pos) if v.m.size == 1 else v.entries()
        if len(vals) != len(pos):
            raise ValueError('assignment size mismatch')
        for (i, j), e in zip(pos, vals):
            self.m[i, j] = e
        if isinstance(v, (SX, MX)) and isinstance(self, DM):
            raise TypeError('symbolic assignment into DM')

    # arithmetic
    def __add__(self, o):
        return _elementwise(_add, self, o)

    def __radd__(self, o):
        return _elementwise(_add, o, self)

    def __sub__(self, o):
        return _elementwise(_sub, self, o)

    def __rsub__(self, o):
        return _elementwise(_sub, o, self)

    def __mul__(self, o):
        return _elementwise(_mul, self, o)

    def __rmul__(self, o):
        return _elementwise(_mul, o, self)

    def __truediv__(self, o):
        return _elementwise(_div, self, o)

    def __rtruediv__(self, o):
        return _elementwise(_div, o, self)

    def __pow__(self, o):
        return _elementwise(_pow, self, o)

    def __rpow__(self, o):
        return _elementwise(_pow, o, self)

    def __neg__(self):
        return _elementwise(_neg, self)

    def __pos__(self):
        return self

    def __matmul__(self, o):
        return mtimes(self, o)

    def __rmatmul__(self, o):
        return mtimes(o, self)

    def __ge__(self, o):
        return _elementwise(_ge, self, o)

    def __gt__(self, o):
        return _elementwise(_gt, self, o)

    def __le__(self, o):
        return _elementwise(_le, self, o)

    def __lt__(self, o):
        return _elementwise(_lt, self, o)

    def __eq__(self, o):
        return _elementwise(_eq, self, o)

    def __ne__(self, o):
        return _elementwise(_ne, self, o)

    # numeric access
    def is_constant(self):
        return all(_num(e) for e in self.m.reshape(-1))

    def __array__(self, dtype=None, copy=None):
        if not self.is_constant():
            raise TypeError('symbolic matrix has no numeric value')
        return np.array(self.m, dtype=dtype or float)

    def full(self):
        return self.__array__()

    def __float__(self):
        return float(_entry(self))

    def __bool__(self):
        e = _entry(self)
        if not _num(e):
            raise TypeError('truth value of a symbolic expression')
        return bool(e != 0)

    def __repr__(self):
        return f'{type(self).__name__}{self.shape}'


class SX(_Mat):
    ''' symbolic matrix (scalar-expression entries) '''


class MX(_Mat):
    ''' symbolic matrix; here the same scalar DAG as SX '''


class DM(_Mat):
    ''' numeric matrix '''


# ------------------------------------------------------------------------------ free functions
def _cat(args, axis):
    ms = [_to_mat(a) for a in args]
    ms = [m for m in ms if m.m.size > 0]
    if not ms:
        return DM._wrap(np.zeros((0, 1) if axis == 0 else (1, 0), dtype=object))
    return _result_cls(*ms)._wrap(np.concatenate([m.m for m in ms], axis=axis))


def vertcat(*args):
    return _cat(args, 0)


def horzcat(*args):
    return _cat(args, 1)


def mtimes(a, b):
    A, B = _to_mat(a), _to_mat(b)
    if A.shape == (1, 1) or B.shape == (1, 1):
        return A * B
    if A.shape[1] != B.shape[0]:
        raise ValueError(f'mtimes dimension mismatch {A.shape} @ {B.shape}')
    out = np.empty((A.shape[0], B.shape[1]), dtype=object)
    for i in range(A.shape[0]):
        for j in range(B.shape[1]):
            acc = 0.0
            for k in range(A.shape[1]):
                acc = _add(acc, _mul(A.m[i, k], B.m[k, j]))
            out[i, j] = acc
    return _result_cls(A, B)._wrap(out)


def _apply(build, x):
    if isinstance(x, (numbers.Number, np.number)):
        return float(build(float(x)))
    return _elementwise(build, x)


def sin(x):
    return _apply(_sin, x)


def cos(x):
    return _apply(_cos, x)


def tan(x):
    return _apply(_tan, x)


def sqrt(x):
    return _apply(_sqrt, x)


def exp(x):
    return _apply(_exp, x)


def log(x):
    return _apply(_log, x)


def dot(a, b):
    A, B = _to_mat(a), _to_mat(b)
    acc = 0.0
    for x, y in zip(A.entries(), B.entries()):
        acc = _add(acc, _mul(x, y))
    return _result_cls(A, B)._wrap(np.array([[acc]], dtype=object))


def norm_2(x):
    return sqrt(dot(x, x))


def cross(a, b):
    A, B = _to_mat(a), _to_mat(b)
    x, y = A.entries(), B.entries()
    out = [_sub(_mul(x[1], y[2]), _mul(x[2], y[1])),
           _sub(_mul(x[2], y[0]), _mul(x[0], y[2])),
           _sub(_mul(x[0], y[1]), _mul(x[1], y[0]))]
    shape = (1, 3) if A.shape[0] == 1 else (3, 1)
    return _result_cls(A, B)._wrap(np.array(out, dtype=object).reshape(shape))


def bilin(A, x, y):
    ''' x' A y over the structural nonzeros of A '''
    M, X, Y = _to_mat(A), _to_mat(x), _to_mat(y)
    xe, ye = X.entries(), Y.entries()
    acc = 0.0
    for j in range(M.shape[1]):
        for i in range(M.shape[0]):
            a = M.m[i, j]
            if _num(a) and a == 0:
                continue
            acc = _add(acc, _mul(_mul(xe[i], a), ye[j]))
    return _result_cls(M, X, Y)._wrap(np.array([[acc]], dtype=object))


def inv(A):
    M = _to_mat(A)
    if M.is_constant():
        return DM._wrap(np.linalg.inv(np.array(M.m, dtype=float)).astype(object))
    n = M.shape[0]
    if n == 1:
        return type(M)._wrap(np.array([[_div(1.0, M.m[0, 0])]], dtype=object))
    if n == 2:
        a, b, c, d = M.m[0, 0], M.m[0, 1], M.m[1, 0], M.m[1, 1]
        det = _sub(_mul(a, d), _mul(b, c))
        out = np.array([[_div(d, det), _div(_neg(b), det)], [_div(_neg(c), det), _div(a, det)]], dtype=object)
        return type(M)._wrap(out)
    raise NotImplementedError('symbolic inverse larger than 2 x 2')


def if_else(c, a, b, *_):
    return _elementwise(_ifelse, c, a, b)


def cumsum(x):
    X = _to_mat(x)
    e = X.entries()
    out, acc = [], None
    for v in e:
        acc = v if acc is None else _add(acc, v)
        out.append(acc)
    return type(X)._wrap(np.array(out, dtype=object).reshape(X.shape))


def pw_const(t, tval, val):
    ''' val[0] + sum_i (val[i+1] - val[i]) * (t >= tval[i]) '''
    T, TV, V = _to_mat(t), _to_mat(tval), _to_mat(val)
    tv, v = TV.entries(), V.entries()
    if len(v) != len(tv) + 1:
        raise ValueError('pw_const: val must have one more entry than tval')
    tt = _entry(T)
    ret = v[0]
    for i in range(len(tv)):
        ret = _add(ret, _mul(_sub(v[i + 1], v[i]), _ge(tt, tv[i])))
    return _result_cls(T, TV, V)._wrap(np.array([[ret]], dtype=object))


def pw_lin(t, tval, val):
    ''' linear segments through (tval, val), extrapolated at both ends '''
    T, TV, V = _to_mat(t), _to_mat(tval), _to_mat(val)
    tv, v = TV.entries(), V.entries()
    n = len(tv)
    tt = _entry(T)
    seg = []
    for i in range(n - 1):
        g = _div(_sub(v[i + 1], v[i]), _sub(tv[i + 1], tv[i]))
        seg.append(_add(v[i], _mul(g, _sub(tt, tv[i]))))
    return pw_const(T, _result_cls(TV)._wrap(np.array(tv[1:n - 1], dtype=object).reshape(-1, 1)),
                    _result_cls(T, TV, V)._wrap(np.array(seg, dtype=object).reshape(-1, 1)))


def jacobian(expr, x):
    E, X = _to_mat(expr), _to_mat(x)
    ee, xe = E.entries(), X.entries()
    out = np.empty((len(ee), len(xe)), dtype=object)
    for j, xs in enumerate(xe):
        if not (isinstance(xs, _N) and xs.op == 'sym'):
            raise ValueError('jacobian: x must be purely symbolic')
        col = _derivative(ee, xs)
        for i, v in enumerate(col):
            out[i, j] = v
    return _result_cls(E, X)._wrap(out)


def low(*_):
    raise NotImplementedError('low() is not part of the transcription path')


def collocation_points(K, scheme='legendre'):
    ''' Gauss-Legendre roots mapped to [0, 1], computed to 40 digits and rounded once '''
    if scheme != 'legendre':
        raise NotImplementedError(scheme)
    import mpmath
    mpmath.mp.dps = 40
    guess, _ = np.polynomial.legendre.leggauss(K)
    roots = [mpmath.findroot(lambda z: mpmath.legendre(K, z), mpmath.mpf(float(g))) for g in guess]
    return [float((r + 1) / 2) for r in sorted(roots)]


# ------------------------------------------------------------------------------ Function
def _as_arg(x):
    if isinstance(x, _Mat):
        return x
    if isinstance(x, (list, tuple)) and all(isinstance(e, (numbers.Number, np.number)) for e in x):
        return DM._wrap(np.array([float(e) for e in x], dtype=object).reshape(-1, 1))
    return _to_mat(x)


class Function:
    ''' inline-substituting function of symbolic inputs '''

    def __init__(self, name, inputs, outputs, *names):
        self.name = name
        self.ins = [_to_mat(i) for i in inputs]
        if isinstance(outputs, _Mat):
            outputs = [outputs]
        self.outs = [_to_mat(o) for o in outputs]
        self.leaf_pos = []
        for k, m in enumerate(self.ins):
            for e in m.entries():
                if not (isinstance(e, _N) and e.op == 'sym'):
                    raise ValueError(f'Function {name}: input {k} is not purely symbolic')
        self._order = None

    def _ordered(self):
        if self._order is None:
            roots = [e for o in self.outs for e in o.entries()]
            self._order = _topo(roots)
        return self._order

    def size_in(self, i):
        return self.ins[i].shape

    def size_out(self, i):
        return self.outs[i].shape

    def n_in(self):
        return len(self.ins)

    def n_out(self):
        return len(self.outs)

    def call(self, args):
        return list(self._call(args))

    def __call__(self, *args):
        out = self._call(list(args))
        return out[0] if len(out) == 1 else tuple(out)

    def _call(self, args):
        if len(args) != len(self.ins):
            raise ValueError(f'Function {self.name}: {len(args)} arguments, {len(self.ins)} inputs')
        mats = [_as_arg(a) for a in args]
        leaf = {}
        for m_in, m_arg in zip(self.ins, mats):
            if m_arg.m.size != m_in.m.size:
                raise ValueError(f'Function {self.name}: argument of shape {m_arg.shape}, input {m_in.shape}')
            for s, v in zip(m_in.entries(), m_arg.entries()):
                leaf[s.id] = v
        numeric = all(m.is_constant() for m in mats)
        order = self._ordered()
        if numeric:
            val = evaluate(order, leaf)
            cls = DM
        else:
            val = _substitute(order, leaf)
            cls = _result_cls(*mats)
            if cls is DM:
                cls = SX
        outs = []
        for o in self.outs:
            a = np.empty(o.shape, dtype=object)
            for i in range(o.shape[0]):
                for j in range(o.shape[1]):
                    e = o.m[i, j]
                    v = val[e.id] if isinstance(e, _N) else e
                    a[i, j] = float(v) if numeric else v
            outs.append(cls._wrap(a))
        return outs


# ------------------------------------------------------------------------------ inert placeholders
class _Integrator:
    def __init__(self, prob):
        self.prob = prob

    def __call__(self, **kw):
        x = _to_mat(self.prob['x'])
        return {'xf': MX.sym('integrator_xf_unevaluated', x.shape)}


def integrator(name, solver, prob, *args, **kw):
    ''' SUNDIALS is not part of the transcription: construction only '''
    return _Integrator(prob)


class _NlpSol:
    def __init__(self, prob, opts):
        self.prob, self.opts = prob, opts

    def __call__(self, **kw):
        raise RuntimeError('stand-in: no IPOPT (the golden generator stops before the solve)')

    def stats(self):
        return {'success': True, 't_wall_nlp_f': 0.0, 't_wall_nlp_g': 0.0, 't_wall_nlp_grad_f': 0.0,
                't_wall_nlp_hess_l': 0.0, 't_wall_nlp_jac_g': 0.0}


def nlpsol(name, plugin, prob, opts=None):
    return _NlpSol(prob, opts or {})
