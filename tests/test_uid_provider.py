"""UIDProvider, after the reference's TestUIDProvider (deeplearning4j-core/src/test/java/org/deeplearning4j/util/
TestUIDProvider.java): the process and hardware ids are non-empty and stable across calls. CPU."""
from deeplearning4j_amd.utils.uid import UIDProvider


def test_uid_provider():
    p, h = UIDProvider.getJVMUID(), UIDProvider.getHardwareUID()
    assert p and h
    assert p == UIDProvider.getJVMUID() == UIDProvider.getProcessUID()
    assert h == UIDProvider.getHardwareUID()
