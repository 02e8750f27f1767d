{{- define "amd-gpu-operator.fullname" -}}
{{- printf "%s-%s" .Release.Name "amd-gpu-operator" | trunc 63 | trimSuffix "-" -}}
{{- end -}}

{{- define "amd-gpu-operator.labels" -}}
app.kubernetes.io/name: amd-gpu-operator
app.kubernetes.io/instance: {{ .Release.Name }}
app.kubernetes.io/version: {{ .Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .Release.Service }}
helm.sh/chart: {{ printf "%s-%s" .Chart.Name .Chart.Version }}
{{- end -}}

{{- define "amd-gpu-operator.image" -}}
{{ .Values.operator.repository }}/{{ .Values.operator.image }}:{{ .Values.operator.version }}
{{- end -}}
