"""Plugin registry (mirror of moduleregister.py:1-21).

YAML configs name classes (`name: IDFlows`, `name: DenseBlock`, ...) and the
trainers resolve them with `Register.get(name)`.  As in the reference, ONE dict
is shared by every Register subclass, keyed by the class __name__, so the
MI355X classes of this package are found under the reference's names.
"""


class Register(object):
    record = dict()

    def __init__(self):
        super().__init__()

    @classmethod
    def register(cls, obj):
        cls.record[obj.__name__] = obj
        return obj

    @classmethod
    def get(cls, key):
        obj = cls.record.get(key, None)
        if obj:
            return obj
        raise Exception(f"Can not find object {key}")
