"""Test operator for the Python operator runtime, in the reference's operator style
(examples/python-operator-dataflow): doubles every integer input on `doubled`, answers bytes
inputs on `length`, and stops on an input `stop`."""
import pyarrow as pa
import pyarrow.compute as pc
from dora import DoraStatus


class Operator:
    def __init__(self):
        self.seen = 0

    def on_event(self, dora_event, send_output):
        if dora_event["type"] != "INPUT":
            return DoraStatus.CONTINUE
        if dora_event["id"] == "stop":
            return DoraStatus.STOP
        value = dora_event["value"]
        self.seen += 1
        if pa.types.is_integer(value.type) and not pa.types.is_uint8(value.type):
            send_output("doubled", pc.multiply(value, 2), dora_event["metadata"])
        else:
            send_output("length", pa.array([len(value), self.seen], type=pa.uint64()),
                        dora_event["metadata"])
        return DoraStatus.CONTINUE
