{{- define "nos.image" -}}
{{ .Values.image.repository }}:{{ .Values.image.tag | default .Chart.AppVersion }}
{{- end -}}

{{- define "nos.labels" -}}
app.kubernetes.io/part-of: nos
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ .Chart.Name }}-{{ .Chart.Version }}
{{- with .Values.commonLabels }}
{{ toYaml . }}
{{- end }}
{{- end -}}

{{- define "nos.gpuMemoryGB" -}}
{{ .Values.amdGpuResourceMemoryGB | default .Values.nvidiaGpuResourceMemoryGB }}
{{- end -}}

{{- define "nos.leaderElection" -}}
leaderElection:
  leaderElect: {{ .enabled }}
  resourceName: {{ .resourceName }}
  resourceNamespace: {{ .namespace }}
  leaderElectionReleaseOnCancel: true
{{- end -}}
