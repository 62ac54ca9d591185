"""Writes tests/data/feeder48.dss: a synthetic 12.47 kV radial feeder with 48
model-1 load phase elements (above the 16-element limit of the fast PF
kernels), made up for this repository's tests (parity unpinned: there is no
OpenDSS here).  A 12-section 3-phase trunk with a wye 3-phase load at every
bus, two delta 3-phase loads, five 1-phase laterals with 1-phase loads, one
fixed-tap 1-phase regulator and one capacitor.

Usage:  python tests/data/make_feeder48.py
"""
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    L = ["! Synthetic radial test feeder, 48 model-1 load phase elements "
         "(tests/data/make_feeder48.py writes this file)",
         "Clear", "Set DefaultBaseFrequency=60", "",
         "New Circuit.Feeder48 basekv=115 pu=1.04 phases=3 bus1=SourceBus",
         "~ Angle=30 MVAsc3=2000 MVASC1=2100", "",
         "New Transformer.Sub Phases=3 Windings=2 XHL=6",
         "~ wdg=1 bus=SourceBus conn=delta kv=115 kva=10000 %r=0.5",
         "~ wdg=2 bus=T0 conn=wye kv=12.47 kva=10000 %r=0.5", "",
         "New Linecode.trunk nphases=3 BaseFreq=60 units=mi",
         "~ rmatrix=(0.30 | 0.10 0.31 | 0.09 0.10 0.30)",
         "~ xmatrix=(0.80 | 0.35 0.82 | 0.30 0.33 0.81)",
         "~ cmatrix=(12.0 | -3.0 11.5 | -2.0 -1.5 11.8)",
         "New Linecode.lat nphases=1 BaseFreq=60 units=mi",
         "~ rmatrix=(0.90) xmatrix=(0.95) cmatrix=(8.0)", ""]
    for b in range(1, 13):
        L.append("New Line.T%d Phases=3 Bus1=T%d.1.2.3 Bus2=T%d.1.2.3 LineCode=trunk Length=%d units=ft"
                 % (b, b - 1, b, 900 + 50 * (b % 4)))
    L.append("")
    for b in range(1, 13):
        kw = 330 + 60 * (b % 5)
        L.append("New Load.W%d Bus1=T%d.1.2.3 Phases=3 Conn=Wye Model=1 kV=12.47 kW=%d kvar=%d"
                 % (b, b, kw, kw // 2))
    L.append("New Load.D6 Bus1=T6.1.2.3 Phases=3 Conn=Delta Model=1 kV=12.47 kW=900 kvar=420")
    L.append("New Load.D10 Bus1=T10.1.2.3 Phases=3 Conn=Delta Model=1 kV=12.47 kW=780 kvar=360")
    for i, (b, ph) in enumerate(((3, 1), (5, 2), (7, 3), (9, 1), (11, 2))):
        L.append("New Line.LAT%d Phases=1 Bus1=T%d.%d Bus2=L%d.%d LineCode=lat Length=1500 units=ft"
                 % (b, b, ph, b, ph))
        L.append("New Load.S%d Bus1=L%d.%d Phases=1 Conn=Wye Model=1 kV=7.2 kW=%d kvar=%d"
                 % (b, b, ph, 260 + 20 * i, 110 + 10 * i))
    # one fixed-tap 1-phase regulator feeding a far lateral, and a capacitor
    L += ["",
          "New Transformer.RegF phases=1 XHL=0.01 kVAs=[1000 1000] Buses=[T12.3 RF.3] kVs=[7.2 7.2] %LoadLoss=0.01",
          "New Line.LRF Phases=1 Bus1=RF.3 Bus2=F1.3 LineCode=lat Length=1200 units=ft",
          "New Load.F1 Bus1=F1.3 Phases=1 Conn=Wye Model=1 kV=7.2 kW=300 kvar=120",
          "New Capacitor.C8 Bus1=T8 phases=3 kVAR=450 kV=12.47",
          "",
          "Set Voltagebases=[115, 12.47]",
          "Transformer.RegF.Taps=[1.0 1.025]",
          "calcv", "Solve"]
    with open(os.path.join(HERE, "feeder48.dss"), "w") as f:
        f.write("\n".join(L) + "\n")


if __name__ == "__main__":
    main()
