import csv,sys,statistics
api=list(csv.DictReader(open(sys.argv[1])))
gl=[int(a['End_Timestamp'])-int(a['Start_Timestamp']) for a in api if a['Function']=='hipGraphLaunch']
gl=gl[len(gl)//3:]
print(sys.argv[1], 'hipGraphLaunch n', len(gl), 'median us', statistics.median(gl)/1e3, 'p10', sorted(gl)[len(gl)//10]/1e3)
