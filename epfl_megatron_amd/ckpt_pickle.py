"""Pickling for checkpoints that the REFERENCE can load (both directions).

The reference pickles its ``args`` Namespace into every checkpoint, and with
it the enum values of ``megatron.model.enums``.  Our enums
have identical names and values but live in ``epfl_megatron_amd.models.enums``;
pickled as-is, a checkpoint written here would ask the reference's unpickler
for a module it does not have.  ``pickle_module`` below is handed to
``torch.save``: a pickler that writes every class of ``REF_NAMES`` under the
reference's module path (``GLOBAL megatron.model.enums PositionEmbeddingType``)
without importing it.  Our own loader maps those names back
(``checkpointing._safe_globals``), so files round-trip both ways.
"""
import pickle
import types

from .models import enums as _enums

REF_NAMES = {e: ("megatron.model.enums", e.__name__) for e in _enums.ALL_ENUMS}


class RefPickler(pickle._Pickler):
    """Pure-Python pickler (``save_global`` is overridable there, not in the C one)."""

    def save_global(self, obj, name=None):
        ref = REF_NAMES.get(obj)
        if ref is None:
            return super().save_global(obj, name)
        module, qualname = ref
        if self.proto >= 4:
            self.save(module)
            self.save(qualname)
            self.write(pickle.STACK_GLOBAL)
        else:
            self.write(pickle.GLOBAL + bytes(module, "utf-8") + b"\n" +
                       bytes(qualname, "utf-8") + b"\n")
        self.memoize(obj)


pickle_module = types.SimpleNamespace(
    Pickler=RefPickler, Unpickler=pickle.Unpickler, load=pickle.load, dump=pickle.dump,
    loads=pickle.loads, dumps=pickle.dumps, HIGHEST_PROTOCOL=pickle.HIGHEST_PROTOCOL,
    DEFAULT_PROTOCOL=pickle.DEFAULT_PROTOCOL, __name__="epfl_megatron_amd.ckpt_pickle")
