"""Host-side request/response model mirror, written after the reference's models.rs tests
(src/models.rs:427-1109).  Each test cites the reference test it mirrors."""
import struct

import pytest

from reductionist_amd.errors import RequestDataValidation
from reductionist_amd.models import RequestData, Response

URL = "http://example.com/bucket/test--operation-min-dtype-uint64--shape-[10, 5, 2]-etc.bin"


def rd(**kw):  # test_utils.rs:7-29 get_test_request_data
    return RequestData(interface_type="s3", url=URL, dtype="int32", **kw)


def invalid(msg, **kw):
    with pytest.raises(RequestDataValidation, match=msg):
        rd(**kw).validate()


def test_required_and_optional_fields_validate():        # models.rs:428-555
    rd().validate()
    rd(byte_order="little", offset=4, size=8, shape=[2, 5, 1], axis=[1, 2], order="C",
       selection=[[1, 2, 3], [4, 5, 6], [1, 1, 1]], filters=[{"id": "shuffle", "element_size": 4}],
       missing={"missing_value": 42}, compression="gzip").validate()


def test_invalid_interface_type():                        # models.rs:571-577
    with pytest.raises(RequestDataValidation, match="interface type must not be empty"):
        RequestData(interface_type="", url=URL, dtype="int32").validate()


def test_field_validators():                              # models.rs:666-722
    invalid("size must be greater than 0", size=0)
    invalid("shape length must be greater than 0", shape=[])
    invalid("shape indices must be greater than 0", shape=[0])
    invalid("selection length must be greater than 0", shape=[1], selection=[])
    invalid("Selection stride must not be equal to zero", shape=[1], selection=[[1, 2, 0]])


@pytest.mark.parametrize("sel,shape", [([1, 0, 1], [1]), ([1, 0, -1], [1]), ([5, 5, 1], [4]), ([-5, 5, 1], [4]),
                                       ([1, 5, 1], [4]), ([1, -5, 1], [4])])
def test_numpy_selection_semantics_are_valid(sel, shape):  # models.rs:724-803
    rd(shape=shape, selection=[sel]).validate()


def test_request_level_validation():                      # models.rs:741-846
    invalid("Raw data size must be a multiple of dtype size in bytes", size=1)
    invalid("Raw data size must be equal to the product of shape indices and dtype size in bytes",
            size=4, shape=[1, 2])
    invalid("Shape and selection must have the same length", shape=[1, 2], selection=[[1, 2, 1]])
    invalid("Selection requires shape to be specified", selection=[[1, 2, 1]])
    invalid("Axis requires shape to be specified", axis=1)
    invalid("Reduction axis must be within shape", shape=[1], axis=1)
    invalid("Reduction axes must be provided in ascending order", shape=[1, 2], axis=[1, 0])
    invalid("Reduction axes contains duplicates", shape=[1, 2], axis=[1, 1])


def test_missing_invalid_value_for_dtype():               # models.rs:905-911
    invalid("Incompatible value 9223372036854775807 for missing", missing={"missing_value": 2 ** 63 - 1})


def test_unknown_field_and_bad_enums():                   # models.rs:631-665, 848-928
    base = {"interface_type": "s3", "url": URL, "dtype": "int32"}
    for bad in ({"foo": 1}, {"dtype": "int8"}, {"byte_order": "middle"}, {"order": "X"},
                {"compression": {"id": "foo"}}, {"filters": [{"id": "foo", "element_size": 4}]},
                {"missing": {"foo": 1}}):
        with pytest.raises(RequestDataValidation):
            RequestData.from_json({**base, **bad})
    with pytest.raises(RequestDataValidation, match="missing field `dtype`"):
        RequestData.from_json({"interface_type": "s3", "url": URL})


def test_json_optional_fields2():                         # models.rs:965-1004
    r = RequestData.from_json({
        "interface_type": "s3", "url": URL, "dtype": "float64", "byte_order": "big", "offset": 4, "size": 8,
        "shape": [2, 5, 10], "axis": 2, "order": "F", "selection": [[1, 2, 3], [4, 5, 6], [7, 8, 9]],
        "compression": {"id": "zlib"}, "filters": [{"id": "shuffle", "element_size": 8}],
        "missing": {"valid_range": [-1.0, 999.0]}, "option_disable_chunk_cache": True,
        "option_shape_as_bytes": True, "option_count_as_bytes": True})
    assert (r.dtype, r.byte_order, r.shape, r.axis, r.order, r.compression) == \
        ("float64", "big", [2, 5, 10], 2, "F", "zlib")
    assert r.selection == [[1, 2, 3], [4, 5, 6], [7, 8, 9]]
    assert r.filters == [{"id": "shuffle", "element_size": 8}] and r.missing == {"valid_range": [-1.0, 999.0]}


@pytest.mark.parametrize("shape_b,count_b", [(False, False), (True, False), (False, True)])
def test_cbor_response(shape_b, count_b):                 # models.rs:1031-1109
    c = Response(b"\x01\x02\x03", "int32", [3, 2, 1], [3, 1, 2], shape_b, count_b).cbor_fields()
    assert c["bytes"] == b"\x01\x02\x03" and c["dtype"] == "int32" and c["byte_order"] == "little"
    if shape_b:
        assert c["shape"] == [] and list(struct.unpack("<3Q", c["shape_as_bytes"])) == [3, 2, 1]
    else:
        assert c["shape"] == [3, 2, 1] and c["shape_as_bytes"] == b""
    if count_b:
        assert c["count"] == [] and list(struct.unpack("<3q", c["count_as_bytes"])) == [3, 1, 2]
    else:
        assert c["count"] == [3, 1, 2] and c["count_as_bytes"] == b""
