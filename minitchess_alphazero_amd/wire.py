"""Wire formats of the reference's distributed loop, so the GPU puppet and
learner interoperate with the reference's learner, puppets and rlweb unchanged.

Episode payload (puppet -> MQTT -> learner), app/base.py:63-69 and app/learner.py:44-54:
    json.dumps({'episode': [InfoRecorder record, ...], 'userid': ..., 'weights_version': ...,
                'minitchess_alphazero_version': ...})
  `episode_payloads` writes the payloads of a whole batch of games natively from the engine's
  packed records (mtaz_records_json, csrc/mtaz_wire.cpp), byte-identical to that json.dumps
  call; `parse_episode_payload` is the learner side's json.loads.

Weights (learner -> HTTP POST -> rlweb -> HTTP GET -> puppets):
    get_weights_dict  {'weights': jsonpickle.encode(state_dict), 'version': '%Y%m%d%H%M%S'}
                      (app/base.py:201-203)
    push_weights body zlib.compress(json.dumps(that dict).encode())  (app/learner.py:86)
    download_weights  json.loads(zlib.decompress(body)); jsonpickle.decode(content['weights'])
                      (app/base.py:31-39)
  jsonpickle is not installed here, so `encode_weights` writes the jsonpickle
  document of a {name: tensor} dict itself: each tensor is the py/reduce of
  torch._utils._rebuild_tensor_v2 over Tensor.__reduce_ex__(2)'s arguments, its storage the
  py/reduce of torch.storage._load_from_bytes over the storage's own legacy torch.save bytes
  (TypedStorage.__reduce__), which jsonpickle's decoder on the reference side turns back into
  the same tensors.  `decode_weights` is NOT jsonpickle.decode: it accepts only that object
  graph (two whitelisted functions, empty backward-hook OrderedDicts, no references) and loads
  each storage with torch.load(weights_only=True); anything else raises ValueError.  Nothing
  in a downloaded blob is ever unpickled or imported.
"""
import base64
import binascii
import collections
import ctypes
import io
import json
import warnings
import zlib

import numpy as np

from . import _lib

TENSOR_FN = 'torch._utils._rebuild_tensor_v2'
STORAGE_FN = 'torch.storage._load_from_bytes'
ORDERED_DICT = 'collections.OrderedDict'


# ---- episodes ----------------------------------------------------------------------------------
def _cstr(x):
    return None if x is None else str(x).encode('utf-8')


def episode_payloads(records, userid, weights_version, version):
    """One MQTT payload (str) per game of `records` (Engine.records() arrays), equal to
    json.dumps({'episode': Engine.episodes()[g], 'userid': userid, 'weights_version':
    weights_version, 'minitchess_alphazero_version': version}) for each game g."""
    c_i32, c_u32, c_u16, c_f32, c_i64 = ctypes.c_int32, ctypes.c_uint32, ctypes.c_uint16, ctypes.c_float, ctypes.c_int64
    plies = np.ascontiguousarray(records['plies'], np.int32)
    pos = np.ascontiguousarray(records['pos'], np.uint32).reshape(-1, 5)
    action = np.ascontiguousarray(records['action'], np.int32)
    k = np.ascontiguousarray(records['k'], np.int32)
    codes = np.ascontiguousarray(records['codes'], np.uint16)
    visits = np.ascontiguousarray(records['visits'], np.uint32)
    reward = np.ascontiguousarray(records['reward'], np.float32)
    n = len(plies)
    P, E = int(plies.sum()), int(k[:int(plies.sum())].sum())
    if len(pos) < P or len(action) < P or len(k) < P or len(reward) < P or len(codes) < E or len(visits) < E:
        raise ValueError('records arrays shorter than the ply / entry counts')
    strs = [_cstr(userid), _cstr(weights_version), _cstr(version)]
    offsets = np.zeros(n + 1, np.int64)
    L = _lib.lib()
    cap = 256 * P + 32 * E + n * (128 + 6 * sum(len(s or b'') for s in strs))
    for _ in range(2):
        buf = ctypes.create_string_buffer(max(cap, 1))
        total = L.mtaz_records_json(n, _lib.ptr(plies, c_i32), _lib.ptr(pos, c_u32), _lib.ptr(action, c_i32),
                                    _lib.ptr(k, c_i32), _lib.ptr(codes, c_u16), _lib.ptr(visits, c_u32),
                                    _lib.ptr(reward, c_f32), strs[0], strs[1], strs[2], buf, cap,
                                    _lib.ptr(offsets, c_i64))
        _lib.check(total)
        if total <= cap:
            raw = buf.raw[:total].decode('ascii')
            return [raw[offsets[g]:offsets[g + 1]] for g in range(n)]
        cap = total
    raise RuntimeError('mtaz_records_json: size changed between calls')


def parse_episode_payload(payload):
    """The learner side (app/learner.py:44): json.loads of one payload."""
    return json.loads(payload)


# ---- weights -----------------------------------------------------------------------------------
def _tensor_node(t):
    import torch
    t = t.detach().cpu()
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        fn, args = t.__reduce_ex__(2)
        if fn is not torch._utils._rebuild_tensor_v2 or len(args) != 6:
            raise ValueError(f'unsupported tensor for the weights wire format: {type(t)} {t.dtype} {t.layout}')
        storage, offset, size, stride, requires_grad, hooks = args
        sfn, (raw,) = storage.__reduce__()
    if f'{sfn.__module__}.{sfn.__name__}' != STORAGE_FN or len(hooks):
        raise ValueError('unsupported storage / backward hooks for the weights wire format')
    return {'py/reduce': [
        {'py/function': TENSOR_FN},
        {'py/tuple': [
            {'py/reduce': [{'py/function': STORAGE_FN},
                           {'py/tuple': [{'py/b64': base64.b64encode(raw).decode('ascii')}]}]},
            int(offset), {'py/tuple': [int(x) for x in size]}, {'py/tuple': [int(x) for x in stride]},
            bool(requires_grad),
            # OrderedDict().__reduce__() as jsonpickle writes it: class, (), state, listitems, dictitems
            {'py/reduce': [{'py/type': ORDERED_DICT}, {'py/tuple': []}, None, None, {'py/tuple': []}]},
        ]}]}


def encode_weights(weights):
    """jsonpickle.encode(weights) for a {name: tensor} dict (the LearnPuppet.weights dict)."""
    return json.dumps({str(k): _tensor_node(v) for k, v in weights.items()})


def _tag(node, tag, n=None):
    if not isinstance(node, dict) or set(node) != {tag}:
        raise ValueError(f'expected a {tag} node')
    v = node[tag]
    if n is not None and (not isinstance(v, list) or len(v) not in (n if isinstance(n, tuple) else (n,))):
        raise ValueError(f'malformed {tag} node')
    return v


def _int(x, what):
    if type(x) is not int or x < 0:
        raise ValueError(f'bad {what}')
    return x


def _empty_hooks(node):
    if node is None:
        return
    if isinstance(node, dict) and node == {'py/object': ORDERED_DICT}:
        return
    red = _tag(node, 'py/reduce')
    if not isinstance(red, list) or not red or _tag(red[0], 'py/type') != ORDERED_DICT:
        raise ValueError('backward hooks must be an empty OrderedDict')
    for extra in red[1:]:
        if extra is not None and _tag(extra, 'py/tuple') != []:
            raise ValueError('backward hooks must be an empty OrderedDict')


def _decode_tensor(node):
    import torch
    red = _tag(node, 'py/reduce', (2,))
    if _tag(red[0], 'py/function') != TENSOR_FN:
        raise ValueError(f'only {TENSOR_FN} is accepted')
    args = _tag(red[1], 'py/tuple', (6, 7))
    sred = _tag(args[0], 'py/reduce', (2,))
    if _tag(sred[0], 'py/function') != STORAGE_FN:
        raise ValueError(f'only {STORAGE_FN} is accepted')
    (b64node,) = _tag(sred[1], 'py/tuple', 1)
    b64 = _tag(b64node, 'py/b64')
    if not isinstance(b64, str):
        raise ValueError('py/b64 must be a string')
    try:
        raw = base64.b64decode(b64, validate=True)
    except binascii.Error as e:
        raise ValueError(f'bad base64 storage: {e}') from None
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        try:
            storage = torch.load(io.BytesIO(raw), weights_only=True)
        except Exception as e:                      # weights-only unpickler refusals, bad zips
            raise ValueError(f'storage bytes refused by the weights-only loader: {type(e).__name__}') from None
        if not isinstance(storage, torch.storage.TypedStorage):
            raise ValueError('storage bytes did not hold a typed storage')
        offset = _int(args[1], 'storage offset')
        size = tuple(_int(x, 'size') for x in _tag(args[2], 'py/tuple'))
        stride = tuple(_int(x, 'stride') for x in _tag(args[3], 'py/tuple'))
        if type(args[4]) is not bool or len(size) != len(stride):
            raise ValueError('bad requires_grad / shape')
        _empty_hooks(args[5])
        if len(args) == 7 and args[6] not in (None, {}):
            raise ValueError('tensor metadata is not accepted')
        if any(s == 0 for s in size):
            need = 0
        else:
            need = offset + 1 + sum((s - 1) * st for s, st in zip(size, stride))
        if need > storage.size():
            raise ValueError('tensor view exceeds its storage')
        t = torch._utils._rebuild_tensor_v2(storage, offset, size, stride, args[4], collections.OrderedDict())
    return t


def decode_weights(s):
    """The {name: tensor} dict of a jsonpickle weights document (see the module docstring)."""
    doc = json.loads(s)
    if not isinstance(doc, dict):
        raise ValueError('weights document must be a JSON object')
    return {k: _decode_tensor(v) for k, v in doc.items()}


def get_weights_dict(weights, version):
    """LearnPuppet.get_weights_dict (app/base.py:201-203)."""
    return {'weights': encode_weights(weights), 'version': version}


def weights_blob(weights_dict):
    """The HTTP body app/learner.py:86 posts to rlweb: zlib(json(get_weights_dict()))."""
    return zlib.compress(json.dumps(weights_dict).encode())


def load_weights_blob(blob):
    """download_weights' body handling (app/base.py:35-37): {'weights': {name: tensor}, 'version'}."""
    content = json.loads(zlib.decompress(blob))
    if not isinstance(content, dict) or not isinstance(content.get('weights'), str):
        raise ValueError("weights blob must hold {'weights': <jsonpickle str>, 'version': ...}")
    content['weights'] = decode_weights(content['weights'])
    return content
