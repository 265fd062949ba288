{{/* Chart name, truncated to the 63-char DNS label limit.  The top-level nameOverride /
     fullnameOverride are the keys the reference helpers read (reference
     templates/_helpers.tpl:5,14-17), so a release installed with --set fullnameOverride=X keeps
     every object name; the per-component keys of values.yaml are a fallback. */}}
{{- define "bgc.name" -}}
{{- default .Chart.Name (.Values.nameOverride | default .Values.controller.nameOverride) | trunc 63 | trimSuffix "-" }}
{{- end }}

{{/* Release-qualified name; the release name alone when it already contains the chart name. */}}
{{- define "bgc.fullname" -}}
{{- $override := .Values.fullnameOverride | default .Values.controller.fullnameOverride }}
{{- if $override }}
{{- $override | trunc 63 | trimSuffix "-" }}
{{- else }}
{{- $name := include "bgc.name" . }}
{{- if contains $name .Release.Name }}
{{- .Release.Name | trunc 63 | trimSuffix "-" }}
{{- else }}
{{- printf "%s-%s" .Release.Name $name | trunc 63 | trimSuffix "-" }}
{{- end }}
{{- end }}
{{- end }}

{{- define "bgc.chart" -}}
{{- printf "%s-%s" .Chart.Name .Chart.Version | replace "+" "_" | trunc 63 | trimSuffix "-" }}
{{- end }}

{{/* Deployment spec.selector: exactly the reference's (name + instance; reference
     templates/deployment.yaml:12-14).  spec.selector is immutable, so anything else would make
     an in-place `helm upgrade` from a reference release fail.  Call with the root context. */}}
{{- define "bgc.deploymentSelector" -}}
app.kubernetes.io/name: {{ include "bgc.name" . }}
app.kubernetes.io/instance: {{ .Release.Name }}
{{- end }}

{{/* Pod labels and the selector of the Service, PDB and DaemonSet. `component` keeps the
     webhook Service on the admission pods only (the reference shared one selector, so its
     Service also routed to the plain-HTTP controller/synchronizer pods: SURVEY Q1).
     Call with (dict "root" $ "component" "x"). */}}
{{- define "bgc.selectorLabels" -}}
{{- if eq .component "node-agent" }}
{{- /* the DaemonSet's pods carry their own name, so the reference-shaped Deployment
       selectors (name + instance only) never match a node-agent pod */}}
app.kubernetes.io/name: {{ printf "%s-node-agent" (include "bgc.name" .root) | trunc 63 | trimSuffix "-" }}
{{- else }}
app.kubernetes.io/name: {{ include "bgc.name" .root }}
{{- end }}
app.kubernetes.io/instance: {{ .root.Release.Name }}
app.kubernetes.io/component: {{ .component }}
{{- end }}

{{- define "bgc.labels" -}}
helm.sh/chart: {{ include "bgc.chart" .root }}
{{ include "bgc.selectorLabels" . }}
app.kubernetes.io/version: {{ .root.Chart.AppVersion | quote }}
app.kubernetes.io/managed-by: {{ .root.Release.Service }}
{{- end }}

{{- define "bgc.authorizedGroups" -}}
{{- join "," .Values.admission.configs.authorized_group_names }}
{{- end }}
