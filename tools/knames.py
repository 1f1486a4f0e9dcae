"""Kernel names from rocprofv3 CSV rows: no return type, namespaces or parameter list (template
arguments kept), e.g. "void pcamd::(anonymous namespace)::k_screen_oz2<8, 2>(…)" → "k_screen_oz2<8, 2>"."""


def kname(raw):
    k = raw.replace("(anonymous namespace)::", "").replace("pcamd::", "").replace("void ", "")
    depth = 0
    for i, ch in enumerate(k):
        depth += ch == "<"
        depth -= ch == ">"
        if ch == "(" and depth == 0:
            return k[:i].strip()
    return k.strip()
