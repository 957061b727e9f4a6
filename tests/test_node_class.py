"""Node.ComputeClass partition and EscapedConstraints (nomad/structs/node_class.go:
31-132), pinned by node_class_test.go:54-246. The hash value itself is
hashstructure's (go.mod: mitchellh/hashstructure v1.0.0) and is not restated;
only the partition matters: which node changes keep the class
and which split it. nomad_amd/structs.Node.compute_class is what the tests,
the bench and the fixture generators hand the engine as ComputedClass."""
import copy

from nomad_amd import synth
from nomad_amd.structs import Constraint, DeviceGroup, escaped_constraints


def _node():
    n = synth.mock_node("12345678-abcd-efab-cdef-123456789abc")
    n.meta["pci-dss"] = "true"
    return n


def test_computed_class_determinism_and_fields():
    # TestNode_ComputedClass (node_class_test.go:54-81)
    n = _node()
    old = n.compute_class()
    assert old and n.compute_class() == old
    n.datacenter = "New DC"
    assert n.compute_class() != old
    old = n.computed_class
    n.devices.append(DeviceGroup("foo", "gpu", "bam", 1, {}))
    assert n.compute_class() != old


def test_computed_class_ignores_id():
    # TestNode_ComputedClass_Ignore (:83-98)
    n = _node()
    old = n.compute_class()
    n.id = "New ID"
    assert n.compute_class() == old


def test_computed_class_ignores_unique_device_attributes():
    # TestNode_ComputedClass_Device_Attr (:100-122)
    n = _node()
    d = DeviceGroup("foo", "gpu", "bam", 1, {"foo": True})
    n.devices.append(d)
    old = n.compute_class()
    d.attributes["unique.bar"] = False
    assert n.compute_class() == old


def test_computed_class_attributes():
    # TestNode_ComputedClass_Attr (:124-168)
    n = _node()
    old = n.compute_class()
    n.attributes["unique.foo"] = "bar"
    assert n.compute_class() == old
    n.attributes["version"] = "New Version"
    assert n.compute_class() != old
    old = n.computed_class
    n.attributes.pop("driver.exec")
    assert n.compute_class() != old


def test_computed_class_meta():
    # TestNode_ComputedClass_Meta (:170-205)
    n = _node()
    old = n.compute_class()
    n.meta["pci-dss"] = "false"
    assert n.compute_class() != old
    old = n.computed_class
    n.meta["unique.foo"] = "ignore"
    assert n.compute_class() == old


def test_computed_class_ignores_non_hashed_fields():
    # HashInclude: only Datacenter, Attributes, Meta, NodeClass and the device
    # identities are hashed; drivers, resources, networks, volumes are not
    n = _node()
    old = n.compute_class()
    m = copy.deepcopy(n)
    m.cpu_shares, m.memory_mb = 64000, 131072
    m.drivers = {}
    m.host_volumes = {"data": False}
    m.name = "another"
    assert m.compute_class() == old
    m.node_class = "other"
    assert m.compute_class() != old


def test_escaped_constraints():
    # TestNode_EscapedConstraints (:207-246): ${unique.node.id} is not an
    # escaping target, so the escaped set is e1, e2
    ne1 = Constraint("${attr.kernel.name}", "linux", "=")
    ne2 = Constraint("${meta.key_foo}", "linux", "<")
    ne3 = Constraint("${node.dc}", "test", "!=")
    e1 = Constraint("${attr.unique.kernel.name}", "linux", "=")
    e2 = Constraint("${meta.unique.key_foo}", "linux", "<")
    e3 = Constraint("${unique.node.id}", "test", "!=")
    got = escaped_constraints([ne1, ne2, ne3, e1, e2, e3])
    assert got == [e1, e2]
    assert got != [ne1, ne2, ne3]
