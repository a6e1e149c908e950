"""Minimal CasADi-SX stand-in, so the reference's model files run unmodified on the engine.

The reference builds its models with CasADi SX expressions (src/plant.py:16-43,
src/force_model/dynamics.py:22-47, src/jerk_model/dynamics.py:22-52) and uses `ca.cos`/`ca.sin`/
`ca.pi` on plain floats in its trajectory generators (force_model/gen_trajectory.py:77-99).
CasADi is not a dependency of the engine: this module implements exactly that surface —

    SX.sym(name, n), vertcat(*e), + - * / ** and unary -, sin cos tan sqrt exp log fabs tanh
    atan2, pi, .shape / .size() / .size1() / .numel(), indexing

— as a small expression DAG that the façade can evaluate numerically. It is what
`drone_attitude_control_amd/shims/casadi` re-exports under the name `casadi`.

The engine needs two things from a model expression:
  * `affine_coefficients(x, u)` -> (A_c, B_c, c_c) for the OCP dynamics (both reference
    controller models are affine; a non-affine model raises NotImplementedError, as the
    engine solves LQ-OCPs);
  * `crazyflie_plant_params(f, x, u)` -> (mass, g) when a simulator is built on the
    reference plant (plant.py:27-35), which the device plant kernel implements.
"""
import math

import numpy as np

pi = math.pi
inf = math.inf

_next_id = [0]


def _new_sym(name):
    _next_id[0] += 1
    return ("sym", _next_id[0], name)


def _const(v):
    return ("const", float(v))


_UNARY = {
    "neg": lambda a: -a, "sin": np.sin, "cos": np.cos, "tan": np.tan, "sqrt": np.sqrt,
    "exp": np.exp, "log": np.log, "fabs": np.abs, "tanh": np.tanh,
}
_BINARY = {
    "add": lambda a, b: a + b, "sub": lambda a, b: a - b, "mul": lambda a, b: a * b,
    "div": lambda a, b: a / b, "pow": lambda a, b: a ** b, "atan2": np.arctan2,
}


class SX:
    """Column vector of scalar expression nodes (CasADi SX, dense column subset)."""
    __array_priority__ = 100   # numpy scalars/arrays on the left defer to SX's reflected ops

    def __init__(self, nodes):
        self._n = list(nodes)

    # ---------------------------------------------------------------- construction
    @staticmethod
    def sym(name, n=1, m=1):
        if m != 1:
            raise NotImplementedError("SX.sym: only column vectors are supported")
        if n == 1:
            return SX([_new_sym(name)])
        return SX([_new_sym(f"{name}_{i}") for i in range(n)])

    @staticmethod
    def zeros(n=1, m=1):
        if m != 1:
            raise NotImplementedError("SX.zeros: only column vectors are supported")
        return SX([_const(0.0)] * n)

    # ---------------------------------------------------------------- shape
    @property
    def shape(self):
        return (len(self._n), 1)

    def size(self):
        return (len(self._n), 1)

    def size1(self):
        return len(self._n)

    def size2(self):
        return 1

    def numel(self):
        return len(self._n)

    def is_symbolic(self):
        return all(nd[0] == "sym" for nd in self._n)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return SX(self._n[i])
        return SX([self._n[i]])

    def __iter__(self):
        raise TypeError("SX is not iterable; index it or use vertcat")

    def __repr__(self):
        return f"SX({len(self._n)}x1)"

    # ---------------------------------------------------------------- arithmetic
    def _bin(self, other, op, reflected=False):
        o = _as_sx(other)
        a, b = (o, self) if reflected else (self, o)
        na, nb = len(a._n), len(b._n)
        if na != nb and 1 not in (na, nb):
            raise ValueError(f"SX dimension mismatch {na} vs {nb}")
        n = max(na, nb)
        return SX([(op, a._n[i if na > 1 else 0], b._n[i if nb > 1 else 0]) for i in range(n)])

    def __add__(self, o):
        return self._bin(o, "add")

    def __radd__(self, o):
        return self._bin(o, "add", True)

    def __sub__(self, o):
        return self._bin(o, "sub")

    def __rsub__(self, o):
        return self._bin(o, "sub", True)

    def __mul__(self, o):
        return self._bin(o, "mul")

    def __rmul__(self, o):
        return self._bin(o, "mul", True)

    def __truediv__(self, o):
        return self._bin(o, "div")

    def __rtruediv__(self, o):
        return self._bin(o, "div", True)

    def __pow__(self, o):
        return self._bin(o, "pow")

    def __rpow__(self, o):
        return self._bin(o, "pow", True)

    def __neg__(self):
        return SX([("neg", a) for a in self._n])

    def __pos__(self):
        return self

    # ---------------------------------------------------------------- engine hooks
    def affine_coefficients(self, x, u):
        """(A, B, c) with self(x, u) == A x + B u + c: c = f(0, 0) and the Jacobian columns by
        forward-mode differentiation at 0 (exact for affine expressions), checked at random
        points."""
        x, u = _as_sx(x), _as_sx(u)
        nx, nu = x.numel(), u.numel()
        f = lambda xv, uv: evaluate(self, {**_bind(x, xv), **_bind(u, uv)})
        zero = {**_bind(x, np.zeros(nx)), **_bind(u, np.zeros(nu))}
        c = f(np.zeros(nx), np.zeros(nu))
        col = lambda sym, i: _jvp(self, zero, {sym._n[i][1]: 1.0})
        A = np.stack([col(x, i) for i in range(nx)], 1) if nx else np.zeros((len(c), 0))
        B = np.stack([col(u, i) for i in range(nu)], 1) if nu else np.zeros((len(c), 0))
        rng = np.random.default_rng(1)
        for _ in range(4):
            xv, uv = rng.normal(size=nx), rng.normal(size=nu)
            if not np.allclose(f(xv, uv), A @ xv + B @ uv + c, rtol=1e-10, atol=1e-10):
                raise NotImplementedError("model dynamics are not affine in (x, u); the engine solves LQ-OCPs")
        return A, B, c


def _as_sx(v):
    if isinstance(v, SX):
        return v
    a = np.asarray(v, dtype=float).ravel()
    return SX([_const(t) for t in a])


def _bind(sym, values):
    vals = np.asarray(values, dtype=float).ravel()
    if not sym.is_symbolic():
        raise ValueError("expected a vector of SX symbols")
    if vals.size != sym.numel():
        raise ValueError(f"expected {sym.numel()} values, got {vals.size}")
    return {nd[1]: float(t) for nd, t in zip(sym._n, vals)}


def evaluate(expr, env):
    """Numeric value of an SX column for symbol values env {symbol id: float}."""
    memo = {}

    def ev(nd):
        key = id(nd)
        if key in memo:
            return memo[key]
        kind = nd[0]
        if kind == "const":
            r = nd[1]
        elif kind == "sym":
            if nd[1] not in env:
                raise ValueError(f"free symbol '{nd[2]}' in expression")
            r = env[nd[1]]
        elif kind in _UNARY:
            r = float(_UNARY[kind](ev(nd[1])))
        else:
            r = float(_BINARY[kind](ev(nd[1]), ev(nd[2])))
        memo[key] = r
        return r

    return np.array([ev(nd) for nd in _as_sx(expr)._n], dtype=float)


_DUNARY = {   # derivative of the unary ops at a
    "neg": lambda a: -1.0, "sin": np.cos, "cos": lambda a: -np.sin(a), "tan": lambda a: 1.0 / np.cos(a) ** 2,
    "sqrt": lambda a: 0.5 / np.sqrt(a), "exp": np.exp, "log": lambda a: 1.0 / a, "fabs": np.sign,
    "tanh": lambda a: 1.0 - np.tanh(a) ** 2,
}


def _jvp(expr, env, tangent):
    """Directional derivative of an SX column at env along tangent {symbol id: dv}."""
    memo = {}

    def ev(nd):
        key = id(nd)
        if key in memo:
            return memo[key]
        kind = nd[0]
        if kind == "const":
            r = (nd[1], 0.0)
        elif kind == "sym":
            r = (env[nd[1]], tangent.get(nd[1], 0.0))
        elif kind in _UNARY:
            a, da = ev(nd[1])
            r = (float(_UNARY[kind](a)), float(_DUNARY[kind](a)) * da if da != 0.0 else 0.0)
        else:
            (a, da), (b, db) = ev(nd[1]), ev(nd[2])
            v = float(_BINARY[kind](a, b))
            if kind == "add":
                d = da + db
            elif kind == "sub":
                d = da - db
            elif kind == "mul":
                d = (da * b if da != 0.0 else 0.0) + (a * db if db != 0.0 else 0.0)
            elif kind == "div":
                d = (da / b if da != 0.0 else 0.0) - (a * db / (b * b) if db != 0.0 else 0.0)
            elif kind == "pow":
                d = (b * a ** (b - 1) * da if da != 0.0 else 0.0) + (v * np.log(a) * db if db != 0.0 else 0.0)
            else:   # atan2(a, b)
                d = (b * da - a * db) / (a * a + b * b) if (da != 0.0 or db != 0.0) else 0.0
            r = (v, float(d))
        memo[key] = r
        return r

    return np.array([ev(nd)[1] for nd in _as_sx(expr)._n], dtype=float)


def vertcat(*args):
    nodes = []
    for a in args:
        if isinstance(a, (list, tuple)):
            nodes += vertcat(*a)._n
        else:
            nodes += _as_sx(a)._n
    return SX(nodes)


def _unary(name, npfn):
    def fn(a):
        if isinstance(a, SX):
            return SX([(name, t) for t in a._n])
        return npfn(a)
    fn.__name__ = name
    return fn


sin = _unary("sin", np.sin)
cos = _unary("cos", np.cos)
tan = _unary("tan", np.tan)
sqrt = _unary("sqrt", np.sqrt)
exp = _unary("exp", np.exp)
log = _unary("log", np.log)
fabs = _unary("fabs", np.abs)
tanh = _unary("tanh", np.tanh)


def atan2(a, b):
    if isinstance(a, SX) or isinstance(b, SX):
        return _as_sx(a)._bin(b, "atan2")
    return np.arctan2(a, b)


def crazyflie_plant_params(f, x, u):
    """(mass, g) if f(x, u) is the reference plant x' = [vx, vz, F sin(th)/m, F cos(th)/m - g]
    with x = [px, pz, vx, vz], u = [th, F] (src/plant.py:27-35); raises otherwise."""
    f, x, u = _as_sx(f), _as_sx(x), _as_sx(u)
    if (f.numel(), x.numel(), u.numel()) != (4, 4, 2):
        raise NotImplementedError("simulator model is not the 2-D Crazyflie plant (src/plant.py)")
    ev = lambda xv, uv: evaluate(f, {**_bind(x, xv), **_bind(u, uv)})
    g = -ev(np.zeros(4), np.zeros(2))[3]
    inv_m = ev(np.zeros(4), np.array([0.0, 1.0]))[3] + g
    if not (inv_m > 0 and np.isfinite(inv_m)):
        raise NotImplementedError("simulator model is not the 2-D Crazyflie plant (src/plant.py)")
    rng = np.random.default_rng(2)
    for _ in range(4):
        xv, uv = rng.normal(size=4), rng.normal(size=2)
        ref = np.array([xv[2], xv[3], uv[1] * np.sin(uv[0]) * inv_m, uv[1] * np.cos(uv[0]) * inv_m - g])
        if not np.allclose(ev(xv, uv), ref, rtol=1e-12, atol=1e-12):
            raise NotImplementedError("simulator model is not the 2-D Crazyflie plant (src/plant.py)")
    return 1.0 / inv_m, g
