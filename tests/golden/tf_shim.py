"""A small torch-backed stand-in for the parts of TensorFlow / Keras 3 that the
reference's src/agents/dqn_agent.py calls (TEST INFRASTRUCTURE ONLY).

TensorFlow 2.19 / Keras 3.9.2 (uv.lock:999-1000, :283-284) are not installed
here, so the reference's DQNAgent cannot run as shipped.  This module installs a
`tensorflow` module whose ops are restated on torch fp32 CPU tensors, so that
the reference's OWN DQNAgent.__init__ / select_action / remember / learn /
update_target_network / replay code (dqn_agent.py:97-151, :246-274, :312-387,
:428-434) executes unchanged: its replay sampling (random.sample on the deque),
z-score, Double-DQN target, one-hot, MSE, GradientTape, apply_gradients,
counter and `% target_update_frequency` control flow are the reference's; only
the tensor primitives below are restatements of the published Keras/TF
semantics:

  Dense            y = act(x @ kernel + bias), kernel [fan_in, fan_out]
  argmax           first maximum on ties (tf.argmax)
  GradientTape     only ops run inside the `with` block are differentiated
                   (ops outside it are computed without a graph, as in TF)
  MeanSquaredError mean over the last axis, then the batch mean
                   (keras/src/losses/losses.py mean_squared_error)
  Huber            0.5 e^2 if |e| <= delta else delta (|e| - 0.5 delta),
                   delta = 1.0 (keras/src/losses/losses.py huber)
  Adam             keras/src/optimizers/adam.py update_step:
                   m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
                   w -= m * alpha / (sqrt(v) + eps),
                   alpha = lr sqrt(1 - b2^t) / (1 - b1^t), constants in f32,
                   sqrt correctly rounded
  reduce_std       population standard deviation

Precision policy.  By default everything is fp32.  After
keras.mixed_precision.set_global_policy("mixed_float16") -- what train.py:61
does at import -- (or "mixed_bfloat16") the Dense layers built afterwards follow
Keras 3's mixed-precision semantics (keras/src/layers/layer.py __call__ input
autocast + AutocastScope; keras/src/layers/core/dense.py call):

  * the layer casts its floating input to the compute dtype (f16 / bf16);
  * each read of a kernel / bias variable inside the call is the variable's
    f32 value cast (round to nearest even) to the compute dtype; the variables
    and Adam's slots stay f32, and the gradient reaching a variable is the
    16-bit gradient of its cast, widened exactly;
  * x @ kernel is tf.matmul on 16-bit operands as TF runs it on a GPU: f32
    products and sums (TF's default f32 compute type for half GEMMs), ONE
    rounding of the result to the compute dtype; its gradient ops
    (MatMulGrad) are the same kind of matmul: dX = dY kernel^T and
    dkernel = X^T dY, each rounded once;
  * + bias is an elementwise 16-bit add (exact sum, one rounding); the bias
    gradient is the reduce_sum of dY over the batch (f32 accumulation, one
    rounding) -- TF's _AddGrad for the broadcast operand;
  * relu and its gradient are exact in 16 bits; the network's output is
    16-bit, so the reference's own tf.argmax (dqn_agent.py:342, :273) sees
    16-bit Q values and its tf.cast(..., tf.float32) (:345, :350) widens them
    (the gradient of that cast rounds dL/dQ to 16 bits).

The loss, the TD target, one_hot and Adam stay f32 (the reference builds
them from f32 tensors).  There is no loss scaling: the reference's custom
loop applies the raw gradients (no LossScaleOptimizer).  What stays unpinned
is TF's f32 summation order inside a matmul / reduction (torch CPU's is used).
"""
import contextlib
import sys
import types

import numpy as np
import torch

_REC = [0]          # >0 while a GradientTape is recording
SUMMARIES = []      # (name, value, step) from tf.summary.* calls
_POLICY = {"compute": None}  # None: float32; torch.float16 / torch.bfloat16 (mixed)
POLICIES = {"float32": None, "mixed_float16": torch.float16, "mixed_bfloat16": torch.bfloat16}


def set_global_policy(policy):
    """keras.mixed_precision.set_global_policy: layers built afterwards use it."""
    _POLICY["compute"] = POLICIES[policy if isinstance(policy, str) else policy.name]


def _t(x, dtype=None):
    if isinstance(x, torch.Tensor):
        return x if dtype is None else x.to(dtype)
    a = np.asarray(x)
    if dtype is None:
        dtype = torch.float32 if a.dtype.kind == "f" else torch.int32 if a.dtype.kind in "iu" else None
    if a.dtype == np.bool_:
        a = a.astype(np.float32)
        dtype = dtype or torch.float32
    return torch.as_tensor(np.ascontiguousarray(a)).to(dtype)


def _graph():
    return torch.enable_grad() if _REC[0] else torch.no_grad()


class Variable:
    def __init__(self, value):
        self.t = torch.tensor(np.asarray(value, np.float32), requires_grad=True)

    def numpy(self):
        return self.t.detach().numpy().copy()

    def assign(self, value):
        with torch.no_grad():
            self.t.copy_(_t(value, torch.float32))


# ------------------------------------------------------------------ keras layers
class _Init:
    """Keras initializers.  Weights are injected with set_weights in the fixture
    generator (TF's RNG stream is not reproducible here), so these only have to
    produce a tensor of the right shape."""
    def __init__(self, kind, seed=0):
        self.kind, self.rng = kind, np.random.RandomState(seed)

    def __call__(self, shape):
        if self.kind == "zeros":
            return np.zeros(shape, np.float32)
        fi, fo = shape
        if self.kind == "he":
            std = np.sqrt(2.0 / fi) / 0.87962566103423978
            return np.clip(self.rng.normal(0, std, shape), -2 * std, 2 * std).astype(np.float32)
        lim = np.sqrt(6.0 / (fi + fo))
        return self.rng.uniform(-lim, lim, shape).astype(np.float32)


class Input:
    def __init__(self, shape, name=None):
        self.shape = shape


class _MatMul16(torch.autograd.Function):
    """tf.matmul of two 16-bit operands with f32 accumulation, rounded once;
    MatMulGrad: dX = dY W^T, dW = X^T dY, the same kind of matmul."""
    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return (x.float() @ w.float()).to(x.dtype)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        gf = g.float()
        gx = (gf @ w.float().T).to(x.dtype) if ctx.needs_input_grad[0] else None
        gw = (x.float().T @ gf).to(w.dtype) if ctx.needs_input_grad[1] else None
        return gx, gw


class _BiasAdd16(torch.autograd.Function):
    """y + b on 16-bit tensors (b broadcast over the batch): exact sum, one
    rounding.  Gradient: dy as is; db = reduce_sum(dy, batch) accumulated in
    f32, rounded once."""
    @staticmethod
    def forward(ctx, y, b):
        return (y.float() + b.float()).to(y.dtype)

    @staticmethod
    def backward(ctx, g):
        return g, g.float().sum(0).to(g.dtype)


class Dense:
    def __init__(self, units, activation=None, kernel_initializer=None, bias_initializer=None,
                 name=None):
        self.units, self.activation = units, activation
        self.kinit = kernel_initializer or _Init("glorot")
        self.binit = bias_initializer or _Init("zeros")
        self.kernel = self.bias = None
        self.compute = _POLICY["compute"]  # the dtype policy in force at construction

    def build(self, fan_in):
        self.kernel = Variable(self.kinit((fan_in, self.units)))
        self.bias = Variable(self.binit((self.units,)))

    def __call__(self, x):
        with _graph():
            cd = self.compute
            if cd is None:
                y = _t(x, torch.float32) @ self.kernel.t + self.bias.t
            else:
                x = _t(x)
                if x.is_floating_point():
                    x = x.to(cd)  # input autocast
                y = _BiasAdd16.apply(_MatMul16.apply(x, self.kernel.t.to(cd)), self.bias.t.to(cd))
            if self.activation == "relu":
                y = torch.relu(y)
            return y if _REC[0] else y.detach()


class Sequential:
    def __init__(self, layers=()):
        self.layers, self.width = [], None
        for l in layers:
            self.add(l)

    def add(self, layer):
        if isinstance(layer, Input):
            self.width = layer.shape[0]
            return
        layer.build(self.width)
        self.width = layer.units
        self.layers.append(layer)

    def __call__(self, x, training=False):
        for l in self.layers:
            x = l(x)
        return x

    @property
    def trainable_variables(self):
        return [v for l in self.layers for v in (l.kernel, l.bias)]

    def get_weights(self):
        return [v.numpy() for v in self.trainable_variables]

    def set_weights(self, ws):
        for v, w in zip(self.trainable_variables, ws):
            v.assign(w)


# ------------------------------------------------------------------ losses / optimizer
class MeanSquaredError:
    def __call__(self, y_true, y_pred):
        with _graph():
            return torch.mean(torch.mean(torch.square(_t(y_pred) - _t(y_true)), dim=-1))


class Huber:
    def __init__(self, delta=1.0):
        self.delta = float(delta)

    def __call__(self, y_true, y_pred):
        with _graph():
            e = _t(y_pred) - _t(y_true)
            ae = torch.abs(e)
            d = torch.tensor(self.delta, dtype=torch.float32)
            half = torch.tensor(0.5, dtype=torch.float32)
            per = torch.where(ae <= d, half * torch.square(e), d * ae - half * torch.square(d))
            return torch.mean(torch.mean(per, dim=-1))


class Adam:
    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.lr, self.b1, self.b2, self.eps = learning_rate, beta_1, beta_2, epsilon
        self.iterations = 0
        self.slots = {}

    def apply_gradients(self, grads_and_vars):
        f = np.float32
        t = f(self.iterations + 1)
        b1p = np.power(f(self.b1), t, dtype=np.float32)
        b2p = np.power(f(self.b2), t, dtype=np.float32)
        alpha = f(f(self.lr) * np.sqrt(f(1) - b2p, dtype=np.float32)) / f(f(1) - b1p)
        c1, c2 = torch.tensor(f(1 - self.b1)), torch.tensor(f(1 - self.b2))
        a, eps = torch.tensor(alpha), torch.tensor(f(self.eps))
        self.last_grads = []  # the gradients of this step (fixture generator reads them)
        with torch.no_grad():
            for g, var in grads_and_vars:
                self.last_grads.append(g.detach().clone())
                m, v = self.slots.setdefault(id(var), (torch.zeros_like(var.t), torch.zeros_like(var.t)))
                m += (g - m) * c1
                v += (torch.square(g) - v) * c2
                # sqrt correctly rounded, as TF's (Eigen's sqrt on CPU and GPU):
                # torch's vectorised f32 CPU sqrt is off by one ulp in ~0.7 %
                # of inputs; the f64 root rounded to f32 is exact
                var.t -= (m * a) / (torch.sqrt(v.double()).float() + eps)
        self.iterations += 1


class GradientTape:
    def __enter__(self):
        _REC[0] += 1
        return self

    def __exit__(self, *exc):
        _REC[0] -= 1
        return False

    def gradient(self, loss, variables):
        return list(torch.autograd.grad(loss, [v.t for v in variables]))


# ------------------------------------------------------------------ tensor ops
def convert_to_tensor(x, dtype=None):
    return _t(x, dtype)


def argmax(x, axis=0, output_type=torch.int64):
    return torch.argmax(_t(x), dim=axis).to(output_type)


def stack(xs, axis=0):
    return torch.stack([_t(x) for x in xs], dim=axis)


def range_(n):
    return torch.arange(n, dtype=torch.int32)


def gather_nd(params, indices):
    p, i = _t(params), _t(indices).long()
    return p[tuple(i[:, k] for k in range(i.shape[1]))]


def cast(x, dtype):
    return _t(x).to(dtype)


def reduce_sum(x, axis=None):
    with _graph():
        return torch.sum(_t(x)) if axis is None else torch.sum(_t(x), dim=axis)


def reduce_mean(x, axis=None):
    with _graph():
        x = _t(x) if _REC[0] else _t(x).detach()
        return torch.mean(x) if axis is None else torch.mean(x, dim=axis)


def reduce_std(x, axis=None):
    x = _t(x).detach()
    return torch.std(x, unbiased=False) if axis is None else torch.std(x, dim=axis, unbiased=False)


def one_hot(idx, depth, dtype=torch.float32):
    return torch.nn.functional.one_hot(_t(idx).long(), depth).to(dtype)


class _Writer:
    @contextlib.contextmanager
    def as_default(self):
        yield


def _scalar(name, value, step=None):
    v = value.detach().numpy() if isinstance(value, torch.Tensor) else np.asarray(value)
    SUMMARIES.append((name, np.array(v, dtype=np.float64), int(step)))


def install():
    """Register the shim as `tensorflow` (and tensorflow.keras*) in sys.modules."""
    tf = types.ModuleType("tensorflow")
    tf.float32, tf.int32, tf.float16 = torch.float32, torch.int32, torch.float16
    tf.bfloat16 = torch.bfloat16
    tf.convert_to_tensor, tf.argmax, tf.stack, tf.range = convert_to_tensor, argmax, stack, range_
    tf.gather_nd, tf.cast, tf.reduce_sum, tf.reduce_mean = gather_nd, cast, reduce_sum, reduce_mean
    tf.one_hot, tf.GradientTape = one_hot, GradientTape
    tf.math = types.SimpleNamespace(reduce_std=reduce_std)
    tf.function = lambda *a, **k: (lambda f: f)
    tf.summary = types.SimpleNamespace(create_file_writer=lambda path: _Writer(),
                                       scalar=_scalar, histogram=_scalar)
    tf.config = types.SimpleNamespace(
        list_physical_devices=lambda kind: [],
        experimental=types.SimpleNamespace(set_memory_growth=lambda g, b: None))
    tf.random = types.SimpleNamespace(set_seed=lambda s: None)
    keras = types.ModuleType("tensorflow.keras")
    keras.Sequential = Sequential
    keras.initializers = types.SimpleNamespace(HeNormal=lambda: _Init("he", 1),
                                               GlorotUniform=lambda: _Init("glorot", 2),
                                               Zeros=lambda: _Init("zeros"))
    layers = types.ModuleType("tensorflow.keras.layers")
    layers.Dense, layers.Input, layers.Concatenate = Dense, Input, object
    keras.layers = layers
    keras.losses = types.SimpleNamespace(MeanSquaredError=MeanSquaredError, Huber=Huber)
    keras.optimizers = types.SimpleNamespace(Adam=Adam)
    keras.mixed_precision = types.SimpleNamespace(set_global_policy=set_global_policy)
    tf.keras = keras
    sys.modules["tensorflow"] = tf
    sys.modules["tensorflow.keras"] = keras
    sys.modules["tensorflow.keras.layers"] = layers
    return tf
