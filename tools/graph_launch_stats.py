"""hipGraphLaunch host cost from a rocprofv3 --hip-trace csv (median and p10 over the
last two thirds of the calls):

    python tools/graph_launch_stats.py gpurun_out/.../run_hip_api_trace.csv
"""
import csv,sys,statistics
api=list(csv.DictReader(open(sys.argv[1])))
gl=[int(a['End_Timestamp'])-int(a['Start_Timestamp']) for a in api if a['Function']=='hipGraphLaunch']
gl=gl[len(gl)//3:]
print(sys.argv[1], 'hipGraphLaunch n', len(gl), 'median us', statistics.median(gl)/1e3, 'p10', sorted(gl)[len(gl)//10]/1e3)
