"""Writes the round-2/3 PrefetchLoader ordering into a copy of prefetch.py (the N = 2 probe's
"old" variant): sample-output buffers from the caller's stream pool, no record_stream.
Usage: python tools/r04_old_loader.py <copy of DistGNN/dataloading/prefetch.py>"""
import sys

path = sys.argv[1]
src = open(path).read()
edits = [
    ("prep = self.sampler._prepare(seeds, self.fan_out, packed=True,\n"
     "                                     alloc_stream=self._ids[w])",
     "prep = self.sampler._prepare(seeds, self.fan_out, packed=True)"),
    ("        if prep[0] is not seeds:\n            prep[0].record_stream(self._streams[w])\n", ""),
    ("            buf.record_stream(self._c_obj)\n", "            pass\n"),
]
for old, new in edits:
    assert src.count(old) == 1, old
    src = src.replace(old, new)
open(path, "w").write(src)
print("old loader ordering written to", path)
