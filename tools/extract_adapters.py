"""Extract the reference's adapter database (porechop_abi/adapters.py:77-463) and the flank
sequences of its full-barcode builders (:466-498) into custom_porechop_abi_amd/data/adapters.json.

Container-only tool (reads /root/reference as text via the ast module; executes nothing from it).
The JSON is input DATA for the engine: set names and nucleotide sequences.
"""
import ast
import json
import os
import sys

REF = sys.argv[1] if len(sys.argv) > 1 else '/root/reference/porechop_abi/adapters.py'
OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   'custom_porechop_abi_amd', 'data', 'adapters.json')

tree = ast.parse(open(REF).read())
sets = []
flanks = {}
for node in tree.body:
    if isinstance(node, ast.Assign) and getattr(node.targets[0], 'id', None) == 'ADAPTERS':
        for call in node.value.elts:
            entry = {'name': ast.literal_eval(call.args[0]), 'start': None, 'end': None, 'both': None}
            for kw in call.keywords:
                v = ast.literal_eval(kw.value)
                key = {'start_sequence': 'start', 'end_sequence': 'end', 'both_ends_sequence': 'both'}[kw.arg]
                entry[key] = list(v) if v else None
            sets.append(entry)
    if isinstance(node, ast.FunctionDef) and node.name.startswith('make_'):
        nodes = [n for n in ast.walk(node)
                 if isinstance(n, ast.Constant) and isinstance(n.value, str) and set(n.value) <= set('ACGT')
                 and len(n.value) >= 4]
        nodes.sort(key=lambda n: (n.lineno, n.col_offset))   # source order
        flanks[node.name] = [n.value for n in nodes]
json.dump({'source': 'porechop_abi/adapters.py (reference @ 2024_08_07)', 'sets': sets,
           'full_barcode_flanks': flanks}, open(OUT, 'w'), indent=1)
print('wrote', OUT, len(sets), 'sets', {k: len(v) for k, v in flanks.items()})
