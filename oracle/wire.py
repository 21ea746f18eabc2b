"""ORACLE (test infrastructure only): CPU restatement of the reference's wire formats, the
checker for minitchess_alphazero_amd/wire.py and csrc/mtaz_wire.cpp.

* episode payload: the reference's own expression, app/base.py:63-69, over InfoRecorder
  records (exp/callbacks.py:40-54).
* jsonpickle (absent here; unpinned in /root/reference: Dockerfile:34 `pip install jsonpickle`,
  no version): its published pickling algorithm restated for the object graph a state_dict
  produces (jsonpickle/pickler.py Pickler._flatten_obj_instance: objects with __reduce_ex__
  / __reduce__ become {"py/reduce": [f, args, state, listitems, dictitems]} with trailing
  None entries trimmed and iterators lifted into tuples; functions {"py/function":
  "module.name"}, classes {"py/type": ...}, tuples {"py/tuple": [...]}, bytes {"py/b64":
  base64}), and its Unpickler for the same tags (jsonpickle/unpickler.py: py/reduce calls
  f(*args) then applies state / listitems / dictitems).  The restore imports only names in
  ALLOWED and is only ever fed documents this repository wrote.
  Parity of the exact jsonpickle bytes is unpinned (no jsonpickle, no fixture in the
  reference); what is pinned is that the reference-side decode semantics rebuild the tensors.
"""
import base64
import importlib
import json
import types
import warnings


def episode_payload(episode, userid, weights_version, version):
    """app/base.py:63-69: the MQTT message for one episode."""
    data = {
        'episode': episode,
        'userid': userid,
        'weights_version': weights_version,
        'minitchess_alphazero_version': version,
    }
    return json.dumps(data)


def _name(obj):
    return f'{obj.__module__}.{obj.__qualname__}'


def jsonpickle_flatten(obj):
    """jsonpickle.encode's flattening (unpicklable=True) for primitives, lists, plain dicts with
    str keys, tuples, bytes, functions, classes and objects that reduce."""
    if obj is None or type(obj) in (str, bool, int, float):
        return obj
    if type(obj) is bytes:
        return {'py/b64': base64.b64encode(obj).decode('ascii')}
    if type(obj) is list:
        return [jsonpickle_flatten(v) for v in obj]
    if type(obj) is dict:
        return {k: jsonpickle_flatten(v) for k, v in obj.items()}
    if type(obj) is tuple:
        return {'py/tuple': [jsonpickle_flatten(v) for v in obj]}
    if isinstance(obj, type):
        return {'py/type': _name(obj)}
    if isinstance(obj, (types.FunctionType, types.BuiltinFunctionType)):
        return {'py/function': _name(obj)}
    cls = type(obj)
    with warnings.catch_warnings():
        warnings.simplefilter('ignore')
        if cls.__reduce_ex__ is not object.__reduce_ex__:
            rv = obj.__reduce_ex__(2)
        else:
            rv = obj.__reduce__()
    rv = list(rv) + [None] * (5 - len(rv))
    for i in (3, 4):
        if rv[i] is not None and not isinstance(rv[i], (list, tuple)):
            rv[i] = tuple(rv[i])
    out = [jsonpickle_flatten(v) for v in rv]
    last = len(out) - 1
    while last >= 2 and out[last] is None:
        last -= 1
    return {'py/reduce': out[:last + 1]}


ALLOWED = {'torch._utils._rebuild_tensor_v2', 'torch.storage._load_from_bytes', 'collections.OrderedDict'}


def _load(name):
    if name not in ALLOWED:
        raise ValueError(f'{name} not allowed in the oracle restore')
    mod, attr = name.rsplit('.', 1)
    return getattr(importlib.import_module(mod), attr)


def jsonpickle_restore(node):
    """jsonpickle.decode's restore for the tags jsonpickle_flatten writes."""
    if isinstance(node, list):
        return [jsonpickle_restore(v) for v in node]
    if not isinstance(node, dict):
        return node
    if 'py/b64' in node:
        return base64.b64decode(node['py/b64'])
    if 'py/tuple' in node:
        return tuple(jsonpickle_restore(v) for v in node['py/tuple'])
    if 'py/function' in node:
        return _load(node['py/function'])
    if 'py/type' in node:
        return _load(node['py/type'])
    if 'py/reduce' in node:
        parts = [jsonpickle_restore(v) for v in node['py/reduce']] + [None] * 5
        f, args, state, listitems, dictitems = parts[:5]
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')
            obj = f(*args)
        if state:
            obj.__setstate__(state) if hasattr(obj, '__setstate__') else obj.__dict__.update(state)
        for v in listitems or ():
            obj.append(v)
        for k, v in dictitems or ():
            obj[k] = v
        return obj
    return {k: jsonpickle_restore(v) for k, v in node.items()}


def jsonpickle_encode(obj):
    return json.dumps(jsonpickle_flatten(obj))


def jsonpickle_decode(s):
    return jsonpickle_restore(json.loads(s))

