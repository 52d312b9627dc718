"""Copy the reference's committed result artifacts used as parity pins into tests/golden/.

Run in the build container (where /root/reference exists).  The files are data written by the
reference's own runs (Experiments/Results/*): input meshes (points/triangles/mask) and energy
traces Ih0/Ih1/Ih2.txt ("t, Ih" rows, 6 significant digits).  Nothing else is copied.
"""
import os
import shutil

REF = "/root/reference/Experiments/Results"
HERE = os.path.dirname(os.path.abspath(__file__))

FILES = [
    "BaseCircle/CircleEx12points.txt", "BaseCircle/CircleEx12triangles.txt", "BaseCircle/CircleEx12mask.txt",
    "BaseCircle/CircleEx24points.txt", "BaseCircle/CircleEx24triangles.txt", "BaseCircle/CircleEx24mask.txt",
    "BaseCircle3D/3DCircleEx6points.txt", "BaseCircle3D/3DCircleEx6triangles.txt",
    "BaseCircle3D/3DCircleEx6mask.txt",
    "Monitor210/Ih0.txt", "Monitor210/Ih1.txt", "Monitor210/points.txt", "Monitor210/triangles.txt",
    "Monitor220/Ih0.txt", "Monitor310/Ih0.txt", "Monitor340/Ih0.txt", "Monitor2160/Ih0.txt",
    "Monitor380/Ih0.txt", "Monitor3160/Ih0.txt",
    "3DMonitor210/Ih0.txt", "3DMonitor310/Ih0.txt", "3DMonitor310/Ih1.txt",
    # method 2 (backwardsEulerStep) traces
    "Monitor220/Ih2.txt", "Monitor320/Ih2.txt", "3DMonitor210/Ih2.txt",
]

if __name__ == "__main__":
    for f in FILES:
        dst = os.path.join(HERE, f)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copyfile(os.path.join(REF, f), dst)
    print("copied", len(FILES), "files")
