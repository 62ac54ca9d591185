"""Parser for the subset of the OpenDSS script language used by PowerGridworld's
feeders (``gridworld/distribution_system/data/ieee_13_dss/IEEE13Nodeckt.dss``).

The reference hands the .dss file to the OpenDSS engine (``opendss.py:36-39``,
``dss.run_command("Redirect ...")``).  Here the script is parsed into a plain
dict (``FeederSpec``) from which ``feeder.py`` builds the 3-phase nodal
admittance matrix natively (``csrc/pgw_feeder.cpp``).

Supported: comments (``!``, ``//``, ``/* */``), ``~``/``more`` continuation,
``Clear``, ``Set``, ``New``/``Edit`` for ``circuit``/``vsource``,
``transformer`` (2 or 3 windings; ``wdg=k`` positional blocks or the array
forms ``buses= conns= kvs= kvas= taps= %rs=``, ``tap=``, ``XHL/XHT/XLT``,
``%loadloss=``, ``numtaps/mintap/maxtap``; 1-phase units, e.g. the IEEE-13
voltage regulators, and centre-tapped secondaries ``bus.1.0`` / ``bus.0.2``),
``linecode``,
``line`` (linecode or r1/x1/r0/x0/c1/c0, ``Switch=y``), ``load`` (models 1-8 with
``CVRwatts``/``CVRvars``/``ZIPV``) and ``capacitor`` (shunt, or series with
``bus2``); ``RegControl`` (automatic tap control in the snap solve's STATIC
control mode, feeder.Feeder.regulators; ``Set Controlmode=OFF`` keeps the DSS
taps fixed);
property assignments ``Class.Name.Prop=value`` (e.g.
``Transformer.Reg1.Taps=[1.0 1.0625]``); ``Redirect`` of further files;
in-line RPN ``(8 1000 /)``; lower-triangular matrices ``(a | b c | ...)``.
Other commands (``calcv``, ``Solve``, ``BusCoords``, ``Show``) are ignored,
``Set Voltagebases`` and ``Set Controlmode`` are kept.
"""
import math
import os
import re

_UNIT_TO_MI = {"mi": 1.0, "kft": 1000.0 / 5280.0, "ft": 1.0 / 5280.0, "km": 1.0 / 1.609344,
               "m": 1.0 / 1609.344, "me": 1.0 / 1609.344, "in": 1.0 / 63360.0,
               "cm": 1.0 / 160934.4, "none": None}


def _strip_comments(text):
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    out = []
    for line in text.splitlines():
        line = line.split("!")[0]
        line = line.split("//")[0]
        out.append(line)
    return out


def _join_continuations(lines):
    cmds = []
    for line in lines:
        s = line.strip()
        if not s:
            continue
        low = s.lower()
        if s.startswith("~") or low.startswith("more ") or low == "more":
            rest = s[1:] if s.startswith("~") else s[4:]
            if cmds:
                cmds[-1] += " " + rest
            continue
        cmds.append(s)
    return cmds


def _tokenize(cmd):
    """Split 'a=b c=(1 2 /) d=[1 | 2 3]' into tokens respecting brackets/quotes."""
    toks, cur, depth, quote = [], "", 0, None
    for ch in cmd:
        if quote:
            cur += ch
            if ch == quote:
                quote = None
            continue
        if ch in "\"'":
            quote = ch
            cur += ch
        elif ch in "([{":
            depth += 1
            cur += ch
        elif ch in ")]}":
            depth -= 1
            cur += ch
        elif ch.isspace() and depth == 0:
            if cur:
                toks.append(cur)
                cur = ""
        else:
            cur += ch
    if cur:
        toks.append(cur)
    # merge "key = value", "key= value" and "key =value" forms
    merged = []
    i = 0
    while i < len(toks):
        t = toks[i]
        if i + 2 < len(toks) + 0 and i + 1 < len(toks) and toks[i + 1] == "=" and i + 2 < len(toks):
            merged.append(t + "=" + toks[i + 2])
            i += 3
        elif t.endswith("=") and i + 1 < len(toks):
            merged.append(t + toks[i + 1])
            i += 2
        elif i + 1 < len(toks) and toks[i + 1].startswith("=") and "=" not in t:
            merged.append(t + toks[i + 1])
            i += 2
        else:
            merged.append(t)
            i += 1
    return merged


def _unwrap(v):
    v = v.strip()
    if len(v) >= 2 and v[0] in "([{\"'" and v[-1] in ")]}\"'":
        return v[1:-1].strip()
    return v


def parse_number(v):
    """Number or in-line RPN expression, e.g. '(8 1000 /)' -> 0.008."""
    s = _unwrap(v)
    parts = s.replace(",", " ").split()
    if len(parts) == 1:
        return float(parts[0])
    stack = []
    for p in parts:
        if p in "+-*/^":
            b, a = stack.pop(), stack.pop()
            ops = {"+": lambda: a + b, "-": lambda: a - b, "*": lambda: a * b,
                   "/": lambda: a / b, "^": lambda: a ** b}
            stack.append(ops[p]())
        elif p.lower() == "sqrt":
            stack.append(math.sqrt(stack.pop()))
        else:
            stack.append(float(p))
    assert len(stack) == 1, v
    return stack[0]


def parse_matrix(v):
    """Lower-triangular '(a | b c | d e f)' -> full symmetric list of lists."""
    rows = [r.replace(",", " ").split() for r in _unwrap(v).split("|")]
    rows = [[float(x) for x in r] for r in rows if r]
    n = len(rows)
    if n == 1 and len(rows[0]) > 1:
        # full matrix in one row (n*n entries) or a single lower-tri row
        vals = rows[0]
        k = int(round(math.sqrt(len(vals))))
        if k * k == len(vals):
            return [vals[i * k:(i + 1) * k] for i in range(k)]
    full = [[0.0] * n for _ in range(n)]
    if all(len(r) == n for r in rows):               # full rows given
        return rows
    for i, r in enumerate(rows):                     # lower triangle
        assert len(r) == i + 1, v
        for j, x in enumerate(r):
            full[i][j] = x
            full[j][i] = x
    return full


def parse_bus(spec, default_nodes):
    """'671.1.2.3' -> ('671', [1,2,3]);  '671' -> ('671', default_nodes)."""
    parts = spec.split(".")
    name = parts[0].lower()
    nodes = [int(p) for p in parts[1:]] if len(parts) > 1 else list(default_nodes)
    return name, nodes


class FeederSpec(dict):
    """Plain-dict description of a feeder (JSON-serialisable)."""


def parse_dss(path, spec=None):
    spec = spec if spec is not None else FeederSpec(
        source=None, transformers=[], linecodes={}, lines=[], loads=[], voltagebases=[],
        base_frequency=60.0, capacitors=[], regcontrols=[], controlmode="static")
    base_dir = os.path.dirname(os.path.abspath(path))
    with open(path) as f:
        cmds = _join_continuations(_strip_comments(f.read()))
    for cmd in cmds:
        toks = _tokenize(cmd)
        verb = toks[0].lower()
        if verb == "redirect" or verb == "compile":
            sub = os.path.join(base_dir, toks[1])
            if os.path.exists(sub):
                parse_dss(sub, spec)
            continue
        if verb == "set":
            for t in toks[1:]:
                if "=" not in t:
                    continue
                k, v = t.split("=", 1)
                k = k.lower()
                if k == "voltagebases":
                    spec["voltagebases"] = [parse_number(x) for x in _unwrap(v).replace(",", " ").split()]
                elif k == "defaultbasefrequency":
                    spec["base_frequency"] = parse_number(v)
                elif k == "controlmode":
                    spec["controlmode"] = v.lower()
            continue
        if verb.count(".") >= 2 and "=" in verb:      # Class.Name.Prop=value
            target, v = toks[0].split("=", 1)
            cls, name, prop = target.rsplit(".", 2)
            extra = [x.split("=", 1) for x in toks[1:] if "=" in x]
            _assign(spec, cls.lower(), name.lower(), [(prop.strip().lower(), v.strip())] +
                    [(k.strip().lower(), val.strip()) for k, val in extra])
            continue
        if verb not in ("new", "edit"):
            continue                                  # calcv, solve, buscoords, clear, show ...
        obj = toks[1]
        if "=" in obj and obj.lower().startswith("object="):
            obj = obj.split("=", 1)[1]
        cls, name = obj.split(".", 1)
        cls = cls.lower()
        props = []
        for t in toks[2:]:
            if "=" in t:
                k, v = t.split("=", 1)
                props.append((k.strip().lower(), v.strip()))
        if verb == "edit":
            _assign(spec, cls, name.lower(), props)
        elif cls in ("circuit", "vsource"):
            _new_source(spec, name, props)
        elif cls == "transformer":
            _new_transformer(spec, name, props)
        elif cls == "linecode":
            _new_linecode(spec, name, props)
        elif cls == "line":
            _new_line(spec, name, props)
        elif cls == "load":
            _new_load(spec, name, props)
        elif cls == "capacitor":
            _new_capacitor(spec, name, props)
        elif cls == "regcontrol":
            spec["regcontrols"].append(dict(name=name.lower(), props=props))
    return spec


# Classes whose Edit / property assignments cannot change the network model
# (meters, monitors, shapes, geometry data the builder never reads).
_EDIT_IGNORED = {"energymeter", "monitor", "loadshape", "growthshape", "tshape", "priceshape",
                 "spectrum", "xycurve", "wiredata", "cndata", "tsdata", "linegeometry", "linespacing"}


def _assign(spec, cls, name, props):
    """Edit / property assignment on an element defined earlier: transformers
    and loads are updated; classes that cannot change the network are ignored;
    any other class (capacitors, lines, sources ...) raises, since silently
    keeping the original element would give a wrong network."""
    if cls == "transformer":
        for t in spec["transformers"]:
            if t["name"] == name:
                _transformer_props(t, props)
                return
        raise ValueError("Edit of undefined transformer %r" % name)
    if cls == "load":
        for ld in spec["loads"]:
            if ld["name"] == name:
                _load_props(ld, props)
                return
        raise ValueError("Edit of undefined load %r" % name)
    if cls == "regcontrol":
        for rc in spec["regcontrols"]:
            if rc["name"] == name:
                rc["props"] = list(rc["props"]) + list(props)
                return
        raise ValueError("Edit of undefined regcontrol %r" % name)
    if cls in _EDIT_IGNORED:
        return
    raise NotImplementedError("Edit / property assignment of %s.%s (%s) is not supported"
                              % (cls, name, ", ".join(k for k, _ in props)))


def _array(v):
    return [x for x in _unwrap(v).replace(",", " ").split() if x]


def _new_capacitor(spec, name, props):
    """OpenDSS Capacitor defaults: 3 phases, wye, 12.47 kV, 1200 kvar; a kvar
    array (several steps) counts as its sum (all steps in)."""
    c = dict(name=name.lower(), bus1=None, bus2=None, phases=3, conn="wye", kv=12.47, kvar=1200.0)
    for k, v in props:
        if k == "bus1":
            c["bus1"] = v
        elif k == "bus2":          # a series capacitor (bus1 -> bus2, phase by phase)
            c["bus2"] = v
        elif k == "phases":
            c["phases"] = int(parse_number(v))
        elif k == "conn":
            c["conn"] = "delta" if v.lower().startswith("d") or v.lower().startswith("l") else "wye"
        elif k == "kv":
            c["kv"] = parse_number(v)
        elif k == "kvar":
            c["kvar"] = sum(parse_number(x) for x in _array(v))
    spec["capacitors"].append(c)


def _new_source(spec, name, props):
    s = dict(name=name.lower(), bus="sourcebus", basekv=115.0, pu=1.0, angle=0.0, phases=3,
             mvasc3=2000.0, mvasc1=2100.0, x1r1=4.0, x0r0=3.0)
    for k, v in props:
        if k == "bus1":
            s["bus"] = v.split(".")[0].lower()
        elif k in ("basekv", "pu", "angle", "mvasc3", "mvasc1", "x1r1", "x0r0"):
            s[k] = parse_number(v)
        elif k == "phases":
            s["phases"] = int(parse_number(v))
    spec["source"] = s


def _new_transformer(spec, name, props):
    """OpenDSS Transformer defaults: 3 phases, 2 windings, XHL 7 %, XHT 35 %,
    XLT 30 %, each winding wye, 1000 kVA, %R 0.2, tap 1."""
    t = dict(name=name.lower(), phases=3, windings=[{}, {}], xhl=7.0, xht=35.0, xlt=30.0, _w=0)
    _transformer_props(t, props)
    for wd in t["windings"]:
        wd.setdefault("conn", "wye")
        wd.setdefault("kva", t["windings"][0].get("kva", 1000.0))
        wd.setdefault("pct_r", 0.2)
        wd.setdefault("tap", 1.0)
    t["windings"][0].setdefault("kva", 1000.0)
    spec["transformers"].append(t)


def _conn(v):
    return "delta" if v.lower().startswith("d") or v.lower().startswith("l") else "wye"


def _transformer_props(t, props):
    w = t.get("_w", 0)
    W = t["windings"]
    for k, v in props:
        if k == "phases":
            t["phases"] = int(parse_number(v))
        elif k == "windings":
            n = int(parse_number(v))
            if n not in (2, 3):
                raise NotImplementedError("transformer %s: %d windings (2 or 3 supported)" % (t["name"], n))
            while len(W) < n:
                W.append({})
            del W[n:]
        elif k == "wdg":
            w = int(parse_number(v)) - 1
            if w >= len(W):
                raise ValueError("transformer %s: wdg=%d beyond windings=%d" % (t["name"], w + 1, len(W)))
        elif k == "bus":
            W[w]["bus"] = v
        elif k == "conn":
            W[w]["conn"] = _conn(v)
        elif k == "kv":
            W[w]["kv"] = parse_number(v)
        elif k == "kva":
            W[w]["kva"] = parse_number(v)
        elif k in ("%r", "%r1"):
            W[w]["pct_r"] = parse_number(v)
        elif k == "tap":
            W[w]["tap"] = parse_number(v)
        elif k in ("xhl", "x12"):
            t["xhl"] = parse_number(v)
        elif k in ("xht", "x13"):
            t["xht"] = parse_number(v)
        elif k in ("xlt", "x23"):
            t["xlt"] = parse_number(v)
        elif k in ("buses", "conns", "kvs", "kvas", "taps", "%rs"):
            key = {"buses": "bus", "conns": "conn", "kvs": "kv", "kvas": "kva", "taps": "tap",
                   "%rs": "pct_r"}[k]
            vals = _array(v)
            if len(vals) > len(W):
                raise ValueError("transformer %s: %s has %d entries for %d windings"
                                 % (t["name"], k, len(vals), len(W)))
            for i, x in enumerate(vals):
                W[i][key] = x if key == "bus" else _conn(x) if key == "conn" else parse_number(x)
        elif k == "%loadloss":
            for wd in W:
                wd["pct_r"] = parse_number(v) / 2.0
        elif k in ("numtaps", "maxtap", "mintap"):       # the regulator's tap range (RegControl)
            t[k] = parse_number(v)
    t["_w"] = w


def _new_linecode(spec, name, props):
    lc = dict(nphases=3, units="none", r1=0.058, x1=0.1206, r0=0.1784, x0=0.4047,
              c1=3.4, c0=1.6, rmatrix=None, xmatrix=None, cmatrix=None)
    for k, v in props:
        if k == "nphases":
            lc["nphases"] = int(parse_number(v))
        elif k == "units":
            lc["units"] = v.lower()
        elif k in ("rmatrix", "xmatrix", "cmatrix"):
            lc[k] = parse_matrix(v)
        elif k in ("r1", "x1", "r0", "x0", "c1", "c0"):
            lc[k] = parse_number(v)
    spec["linecodes"][name.lower()] = lc


def _new_line(spec, name, props):
    ln = dict(name=name.lower(), phases=3, bus1=None, bus2=None, linecode=None,
              length=1.0, units="none", switch=False)
    seq = {}
    for k, v in props:
        if k == "phases":
            ln["phases"] = int(parse_number(v))
        elif k in ("bus1", "bus2"):
            ln[k] = v
        elif k == "linecode":
            ln["linecode"] = v.lower()
        elif k == "length":
            ln["length"] = parse_number(v)
        elif k == "units":
            ln["units"] = v.lower()
        elif k == "switch":
            ln["switch"] = v.lower().startswith("y") or v.lower().startswith("t")
            if ln["switch"]:
                # OpenDSS Line 'Switch=yes' defaults: r1=x1=r0=x0=1 ohm, c1=1.1, c0=1 nF, length 0.001
                seq.update(r1=1.0, x1=1.0, r0=1.0, x0=1.0, c1=1.1, c0=1.0)
                ln["length"] = 0.001
                ln["units"] = "none"
        elif k in ("r1", "x1", "r0", "x0", "c1", "c0"):
            seq[k] = parse_number(v)
    if seq:
        ln["sequence"] = dict(dict(r1=0.058, x1=0.1206, r0=0.1784, x0=0.4047, c1=3.4, c0=1.6), **seq)
    spec["lines"].append(ln)


def _new_load(spec, name, props):
    ld = dict(name=name.lower(), bus1=None, phases=3, conn="wye", model=1, kv=12.47,
              kw=10.0, kvar=5.0, vminpu=0.95, vmaxpu=1.05, vlowpu=0.50, cvrwatts=1.0, cvrvars=2.0,
              zipv=None)
    _load_props(ld, props)
    spec["loads"].append(ld)


def _load_props(ld, props):
    for k, v in props:
        if k == "bus1":
            ld["bus1"] = v
        elif k == "phases":
            ld["phases"] = int(parse_number(v))
        elif k == "conn":
            ld["conn"] = "delta" if v.lower().startswith("d") or v.lower().startswith("l") else "wye"
        elif k == "model":
            ld["model"] = int(parse_number(v))
        elif k in ("kv", "kw", "kvar", "vminpu", "vmaxpu", "vlowpu", "cvrwatts", "cvrvars"):
            ld[k] = parse_number(v)
        elif k == "zipv":          # [Zp Ip Pp Zq Iq Pq Vcutoff]
            ld["zipv"] = [parse_number(x) for x in _array(v)]
